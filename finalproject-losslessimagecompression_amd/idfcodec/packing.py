"""Host-side weight packing of a DenseBlock (nnblock.py:24-56) for the HIP kernels.

The feature buffer of a DenseBlock is pixel-major with *padded* channel
segments: the block input (a channels) occupies columns [0, a_pad), layer i's
growth (g_i channels, g_i = (i+1)G//d - iG//d, nnblock.py:44) occupies
[a_pad + i*g_pad, a_pad + i*g_pad + g_i), and the padding columns are always
zero.  k_in[i] = a_pad + i*g_pad is the padded width layer i reads.  Weights are
scattered into that padded coordinate system with zeros elsewhere, so every
GEMM has K a multiple of 4, unmasked weight tiles, and padded outputs of 0.

Pure numpy: runs (and is tested) without a GPU.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


def round_up(v: int, m: int) -> int:
    return ((v + m - 1) // m) * m


def tile_n(n: int) -> int:
    """Output-column tile of the GEMM kernels (must match flow_kernels.hip tile_n)."""
    if n <= 16:
        return 16
    if n <= 32:
        return 32
    if n <= 48:
        return 48
    if n <= 64:
        return 64
    w64 = round_up(n, 64) - n
    w128 = round_up(n, 128) - n
    return 128 if w128 <= w64 + 32 else 64


def growths(growth_channel: int, depth: int) -> list[int]:
    """nnblock.py:43-46."""
    return [(i + 1) * growth_channel // depth - i * growth_channel // depth for i in range(depth)]


@dataclass
class BlockGeometry:
    a: int                 # block input channels
    depth: int
    growth: list[int]
    n_head: int
    a_pad: int = 0
    g_pad: int = 0
    k_in: list[int] = field(default_factory=list)

    def __post_init__(self):
        self.a_pad = round_up(self.a, 4)
        self.g_pad = round_up(max(self.growth) if self.growth else 4, 4)
        self.k_in = [self.a_pad + i * self.g_pad for i in range(self.depth + 1)]

    @property
    def width(self) -> int:
        """padded channels of the full feature buffer"""
        return self.k_in[self.depth]

    @property
    def ld_feat(self) -> int:
        return round_up(self.width, 16)

    def pos(self, ch: int) -> int:
        """padded column of logical channel `ch` of the concatenated features"""
        if ch < self.a:
            return ch
        r = ch - self.a
        for j, g in enumerate(self.growth):
            if r < g:
                return self.a_pad + j * self.g_pad + r
            r -= g
        raise IndexError(ch)

    def positions(self, n: int) -> np.ndarray:
        return np.array([self.pos(c) for c in range(n)], dtype=np.int64)

    def flops_per_pixel(self, fold: bool = False) -> int:
        """algorithmic FLOPs of the block per pixel (unpadded).  fold=False: as the
        reference computes it; fold=True: with each 1x1 folded into its 3x3."""
        f = 0
        c = self.a
        for g in self.growth:
            f += (0 if fold else 2 * c * c) + 2 * 9 * c * g
            c += g
        return f + 2 * c * self.n_head


@dataclass
class PackedBlock:
    geom: BlockGeometry
    act: str
    slope: float
    fold: bool
    vtap: list           # fold: [9][g_alloc] per-tap 1x1 bias through W3 (else empty)
    bfull: list          # fold: [g_alloc] b3 + sum_tap vtap (fp32, tap order)
    w1: list[np.ndarray]
    b1: list[np.ndarray]
    w3: list[np.ndarray]
    b3: list[np.ndarray]
    wh: np.ndarray
    bh: np.ndarray
    g_alloc: int
    n1_alloc: list[int]
    ldw1: list[int]
    ldw3: list[int]
    nh_alloc: int
    ldwh: int
    wino_u: list = field(default_factory=list)  # fold+wino: wino_weights() per layer
    wb16: list = field(default_factory=list)    # fold+bf16: bf16_weights() per layer (uint16)
    wx3_u: list = field(default_factory=list)   # fold+wino+wx3: wino_weights_x3() per layer
    wx3_yscale: list = field(default_factory=list)
    dx3_w: list = field(default_factory=list)    # fold+dx3: dx3_weights() per layer (uint16)
    dx3_yscale: list = field(default_factory=list)
    dxb_w: list = field(default_factory=list)    # fold+bf16: dxb_weights() per layer (uint16)


def fold_layer(w1, b1, w3):
    """Fold a DenseLayer's 1x1 conv into its 3x3 conv (nnlayer.py:42-51).

    conv3x3(pad0(W1 x + b1)) = sum_tap W3[tap] W1 x[nbr] + sum_{tap in image} W3[tap] b1,
    exactly, because the reference zero-pads the 1x1 OUTPUT.  Returns
    wf[g, tap, c] = sum_o W3[g, o, tap] W1[o, c] and v[tap, g] = sum_o W3[g, o, tap] b1[o],
    both formed in float64 and rounded once to float32."""
    wf, v = fold_layer64(w1, b1, w3)
    return wf.astype(np.float32), v.astype(np.float32)


def fold_layer64(w1, b1, w3):
    """fold_layer before the final rounding (float64)."""
    w3t = w3.reshape(w3.shape[0], w3.shape[1], 9).astype(np.float64)      # [g, o, tap]
    wf = np.einsum("got,oc->gtc", w3t, w1.astype(np.float64))
    v = np.einsum("got,o->tg", w3t, b1.astype(np.float64))
    return wf, v


# Winograd F(2x2, 3x3) weight transform (Lavin & Gray): U = G g G^T
WINO_G = np.array([[1.0, 0.0, 0.0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0.0, 0.0, 1.0]])


def wino_transform64(w: np.ndarray, nslab: int) -> np.ndarray:
    """U = G g G^T in float64 for every (n, c): [16 positions][n_alloc][nslab*16], from
    w: [n_alloc, 9, ldw] 3x3 weights in the padded channel coordinates."""
    n_alloc = w.shape[0]
    assert n_alloc % 16 == 0
    C = nslab * 16
    g = np.zeros((n_alloc, C, 3, 3), np.float64)
    cw = min(C, w.shape[2])
    g[:, :cw] = w[:, :, :cw].astype(np.float64).transpose(0, 2, 1).reshape(n_alloc, cw, 3, 3)
    return np.einsum("ai,ncij,bj->abnc", WINO_G, g, WINO_G).reshape(16, n_alloc, C)


def wino_weights(w: np.ndarray, nslab: int, U: np.ndarray | None = None) -> np.ndarray:
    """w: [n_alloc, 9, ldw] (float64 preferred) 3x3 weights in the padded channel
    coordinates.  Returns U = G g G^T for every (n, c), rounded once to fp32 and laid out
    in MFMA fragment order [16 positions][nslab][nft][64 lanes][4] (lane = 16*h + r holds
    U[pos][16*f + r][16*slab + 4*h .. +3]) -- what conv3_wino.hip streams per wave."""
    if U is None:
        U = wino_transform64(w, nslab)
    n_alloc = U.shape[1]
    nft = n_alloc // 16
    U = U.reshape(16, nft, 16, nslab, 4, 4)          # pos, f, r, slab, h, e
    U = U.transpose(0, 3, 1, 4, 2, 5)                 # pos, slab, f, h, r, e
    return np.ascontiguousarray(U.reshape(16, nslab, nft, 64, 4).astype(np.float32))


def wino_weights_x3(w: np.ndarray, nslab: int, U: np.ndarray | None = None):
    """Split-f16 form of wino_weights for idf_conv3x3_wx3 (conv3_wino.hip, X3).

    U = G g G^T in float64, scaled by 2^k (k per layer: max |U| * 2^k in [2^14, 2^15), so
    the f16 pairs keep full precision down to ~2^-17 of the largest weight), then split
    Uh = f16(U'), Ul = f16(U' - Uh) (both round-to-nearest-even).  Returns
    (uint16 [16 positions][nslab][nft][64 lanes][8] = (Uh[4], Ul[4]) of the same lane
    element order as wino_weights, yscale = 2^-k)."""
    if U is None:
        U = wino_transform64(w, nslab)
    n_alloc = U.shape[1]
    nft = n_alloc // 16
    k = x3_scale(U)
    Us = U * (2.0 ** k)
    hi = Us.astype(np.float16)
    lo = (Us - hi.astype(np.float64)).astype(np.float16)
    out = np.empty((16, nft, 16, nslab, 4, 2, 4), np.uint16)  # pos, f, r, slab, h, hi/lo, e
    out[..., 0, :] = hi.view(np.uint16).reshape(16, nft, 16, nslab, 4, 4)
    out[..., 1, :] = lo.view(np.uint16).reshape(16, nft, 16, nslab, 4, 4)
    out = out.transpose(0, 3, 1, 4, 2, 5, 6)  # pos, slab, f, h, r, hi/lo, e
    return np.ascontiguousarray(out.reshape(16, nslab, nft, 64, 8)), float(2.0 ** -k)


def x3_scale(U: np.ndarray) -> int:
    """k of the split-f16 pairs: max |U| * 2^k in [2^14, 2^15) (clamped), so the pairs keep full
    precision down to ~2^-17 of the largest weight."""
    m = float(np.abs(U).max())
    k = 0 if m == 0.0 else int(np.floor(np.log2(16384.0 / m)))
    return max(-14, min(k, 60))


def dx3_groups(n_alloc: int):
    """(fragments per group, groups) of a dx3 layer with n_alloc (a multiple of 16) outputs:
    one kernel block computes up to 4 fragments of 16 outputs (conv3_dx3.hip dx3_plan)."""
    nft = max(1, n_alloc // 16)
    nf = min(nft, 4)
    return nf, (nft + nf - 1) // nf


def dx3_weights(w: np.ndarray, C: int):
    """Split-f16 direct-conv weights for idf_conv3x3_dx3 (conv3_dx3.hip).

    w: [n_alloc, 9, ldw] folded 3x3 weights (float64 preferred) in the padded channel
    coordinates, C = the layer's padded input channels.  Scaled by 2^k (x3_scale: max |w| 2^k
    in [2^14, 2^15)) and split wh = f16(w'), wl = f16(w' - wh), both round-to-nearest-even.
    Returns (uint16 [nslab][ngroup][2: hi, lo][9 taps][nf][16 out][16 ch], yscale = 2^-k): per
    slab and output group the A-operand (output-row) fragments one kernel block stages into LDS
    verbatim; channels at or past C are zero.  nf = min(n_alloc / 16, 4) fragments per group,
    ngroup = ceil(n_alloc / 16 / nf) groups (dx3_groups; outputs past n_alloc are zero)."""
    n_alloc = w.shape[0]
    assert n_alloc % 16 == 0
    nf, ngroup = dx3_groups(n_alloc)
    nft = nf * ngroup
    nslab = (C + 15) // 16
    wp = np.zeros((nft * 16, 9, nslab * 16), np.float64)
    cw = min(C, w.shape[2])
    wp[:n_alloc, :, :cw] = w[:, :, :cw]
    k = x3_scale(wp)
    ws = wp * (2.0 ** k)
    hi = ws.astype(np.float16)
    lo = (ws - hi.astype(np.float64)).astype(np.float16)
    out = np.empty((nslab, ngroup, 2, 9, nf, 16, 16), np.uint16)
    for t, part in enumerate((hi, lo)):
        p = part.view(np.uint16).reshape(ngroup, nf, 16, 9, nslab, 16)  # g, f, r, tap, slab, c
        out[:, :, t] = p.transpose(4, 0, 3, 1, 2, 5)
    # The kernel's invariant (conv3_dx3.hip, "split copy"): a layer reads its input's last slab
    # up to the next multiple of 16 channels, i.e. also channels [C, 16 nslab) that other
    # blocks of the same launch are writing (its own outputs).  Those channels must meet
    # exactly +0 weights (hi and lo), so any finite value there adds exactly +-0.
    assert C % 16 == 0 or not out[-1, ..., C % 16:].any(), "dx3 weights past C not zero"
    return np.ascontiguousarray(out), float(2.0 ** -k)


def bf16_weights(w: np.ndarray, C: int) -> np.ndarray:
    """w: [n_alloc][9][ldw] fp32 folded 3x3 weights (padded coordinates), C = the layer's
    padded input channels.  Returns uint16 bf16 bits (round to nearest even) in the fragment
    order of conv3_bf16.hip: [ceil(C/32) slabs][9 taps][4 k-blocks][n_alloc][8 channels]."""
    import torch
    n_alloc = w.shape[0]
    nslab = (C + 31) // 32
    g = np.zeros((n_alloc, 9, nslab * 32), np.float32)
    cw = min(w.shape[2], C)
    g[:, :, :cw] = w[:, :, :cw]
    b = torch.from_numpy(g).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    b = b.reshape(n_alloc, 9, nslab, 4, 8).transpose(2, 1, 3, 0, 4)  # slab, tap, kb, n, e
    return np.ascontiguousarray(b)


def dxb_weights(w: np.ndarray, C: int) -> np.ndarray:
    """bf16 direct-conv weights for idf_conv3x3_dxb (conv3_dx3.hip, bf16 kernel).

    w: [n_alloc <= 48][9][ldw] fp32 folded 3x3 weights (padded coordinates), C = the layer's
    padded input channels.  Returns uint16 bf16 bits (round to nearest even, the values
    bf16_weights holds) as [nslab = ceil(C/16)][9 taps][nf][16 out][16 ch] per slab, each slab
    zero-padded to whole KiB (the kernel's 1-KiB DMA pieces): the A-operand fragments one kernel
    block stages into LDS verbatim.  Channels at or past C are zero (the kernel reads the last
    slab up to the next multiple of 16, where its own outputs land)."""
    import torch
    n_alloc = w.shape[0]
    assert n_alloc % 16 == 0 and n_alloc <= 48
    nf = n_alloc // 16
    nslab = (C + 15) // 16
    g = np.zeros((n_alloc, 9, nslab * 16), np.float32)
    cw = min(w.shape[2], C)
    g[:, :, :cw] = w[:, :, :cw]
    b = torch.from_numpy(g).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    b = b.reshape(nf, 16, 9, nslab, 16).transpose(3, 2, 0, 1, 4)  # slab, tap, f, r, c
    per = 9 * nf * 256                                             # elements of a slab
    pad = (per * 2 + 1023) // 1024 * 1024 // 2
    out = np.zeros((nslab, pad), np.uint16)
    out[:, :per] = b.reshape(nslab, per)
    assert C % 16 == 0 or not b[-1, ..., C % 16:].any(), "dxb weights past C not zero"
    return np.ascontiguousarray(out)


def interior_bias(b3: np.ndarray, v: np.ndarray) -> np.ndarray:
    """b3 + v[0] + ... + v[8], sequential fp32 adds: the order the device's border
    loop uses, so interior and border pixels see the same arithmetic."""
    s = b3.astype(np.float32).copy()
    for t in range(9):
        s = (s + v[t]).astype(np.float32)
    return s


def pack_dense_block(sd: dict, prefix: str, depth: int, act: str = "ReLU",
                     slope: float = 0.01, fold: bool = False, wino: bool = False,
                     bf16: bool = False, wx3: bool = False, dx3: bool = False,
                     dx3_cmax: int | None = None) -> PackedBlock:
    """Pack the reference DenseBlock parameters found under `prefix` in `sd`
    (keys `{prefix}layers.{i}.layers.{0,1}.{weight,bias}`, head `{prefix}layers.{depth}.*`).
    fold=True folds each layer's 1x1 conv into its 3x3 conv (fold_layer); dx3=True also packs
    the split-f16 direct-conv weights (dx3_weights) of the folded layers whose 16-padded input
    width is at most dx3_cmax (None: every layer) -- a prefix of the block, since the input
    widens layer by layer; the remaining layers run on wx3 (flow_kernels.hip dense_block_run)."""
    def arr(k):
        v = sd[prefix + k]
        if hasattr(v, "detach"):
            v = v.detach().cpu().numpy()
        return np.asarray(v, dtype=np.float32)

    w10 = arr("layers.0.layers.0.weight")
    a = int(w10.shape[1])
    gs = [int(arr(f"layers.{i}.layers.1.weight").shape[0]) for i in range(depth)]
    wh_src = arr(f"layers.{depth}.weight")
    n_head = int(wh_src.shape[0])
    geom = BlockGeometry(a=a, depth=depth, growth=gs, n_head=n_head)
    g_alloc = round_up(geom.g_pad, tile_n(geom.g_pad))
    w1s, b1s, w3s, b3s, n1s, ld1s, ld3s = [], [], [], [], [], [], []
    vts, bfs, wus, wbs, wxs, wys, wds, wdy, wdbs = [], [], [], [], [], [], [], [], []
    c = a
    for i in range(depth):
        k = geom.k_in[i]
        pos = geom.positions(c)
        w1 = arr(f"layers.{i}.layers.0.weight")[:, :, 0, 0]  # [c, c]
        b1 = arr(f"layers.{i}.layers.0.bias")
        w3 = arr(f"layers.{i}.layers.1.weight")             # [g, c, 3, 3]
        b3 = arr(f"layers.{i}.layers.1.bias")
        assert w1.shape == (c, c) and w3.shape[1] == c, (w1.shape, w3.shape, c)
        n1_alloc = round_up(k, tile_n(k))
        ldw1 = round_up(k, 16)
        w1p = np.zeros((n1_alloc, ldw1), np.float32)
        w1p[np.ix_(pos, pos)] = w1
        b1p = np.zeros(n1_alloc, np.float32)
        b1p[pos] = b1
        ldw3 = round_up(k, 16)
        w3p = np.zeros((g_alloc, 9, ldw3), np.float32)
        g = w3.shape[0]
        b3p = np.zeros(g_alloc, np.float32)
        b3p[:g] = b3
        if fold:
            wf64, v64 = fold_layer64(w1, b1, w3)
            wf, v = wf64.astype(np.float32), v64.astype(np.float32)
            w3p[:g][:, :, pos] = wf
            if wino or dx3:
                w64 = np.zeros((g_alloc, 9, ldw3), np.float64)
                w64[:g][:, :, pos] = wf64
            if dx3 and (dx3_cmax is None or k <= dx3_cmax):
                wd, yd = dx3_weights(w64, k)
                wds.append(wd)
                wdy.append(yd)
            if wino:
                U64 = wino_transform64(w64, ldw3 // 16)
                wus.append(wino_weights(w64, ldw3 // 16, U64))
                if wx3:
                    ux, ysc = wino_weights_x3(w64, ldw3 // 16, U64)
                    wxs.append(ux)
                    wys.append(ysc)
            if bf16:
                if g_alloc > 48:
                    raise NotImplementedError(
                        f"bf16 DenseLayer convs take growth <= 48 per layer (conv3_bf16.hip: "
                        f"one 48-output tile per block); this layer grows by {g}")
                wbs.append(bf16_weights(w3p, k))
                wdbs.append(dxb_weights(w3p, k))
            vp = np.zeros((9, g_alloc), np.float32)
            vp[:, :g] = v
            vts.append(vp)
            bfs.append(interior_bias(b3p, vp))
        else:
            # [g, c, ky, kx] -> [g, tap=ky*3+kx, pos(c)]
            w3p[:g][:, :, pos] = w3.reshape(g, c, 9).transpose(0, 2, 1)
        w1s.append(w1p); b1s.append(b1p); w3s.append(w3p); b3s.append(b3p)
        n1s.append(n1_alloc); ld1s.append(ldw1); ld3s.append(ldw3)
        c += g
    kh = geom.k_in[depth]
    ldwh = round_up(kh, 16)
    nh_alloc = round_up(n_head, tile_n(n_head))
    whp = np.zeros((nh_alloc, ldwh), np.float32)
    whp[:n_head][:, geom.positions(c)] = wh_src[:, :, 0, 0]
    bhp = np.zeros(nh_alloc, np.float32)
    bhp[:n_head] = arr(f"layers.{depth}.bias")
    return PackedBlock(geom, act, slope, fold, vts, bfs, w1s, b1s, w3s, b3s, whp, bhp, g_alloc,
                       n1s, ld1s, ld3s, nh_alloc, ldwh, wus, wbs, wxs, wys, wds, wdy, wdbs)


# Packing a DenseBlock (float64 folds, Winograd / split / bf16 weight forms) costs ~0.4-1 s of
# host time; an engine packs 27 of them for imagenet64.  Engines built from the same weights
# (a test session building one seeded model many times, an encoder and a decoder in one
# process) share the packed arrays: keyed by the block's parameter bytes and the packing
# arguments, never mutated after packing.  IDF_PACK_CACHE=0 turns it off.
_PACK_CACHE: "collections.OrderedDict" = None
PACK_CACHE_MAX = 96


def pack_dense_block_cached(sd: dict, prefix: str, depth: int, act: str = "ReLU", **kw):
    """pack_dense_block, memoised on the content of the block's parameters under `prefix`."""
    import collections
    import hashlib
    import os
    global _PACK_CACHE
    if os.environ.get("IDF_PACK_CACHE", "1") == "0":
        return pack_dense_block(sd, prefix, depth, act, **kw)
    if _PACK_CACHE is None:
        _PACK_CACHE = collections.OrderedDict()
    h = hashlib.blake2b(digest_size=20)
    for k in sorted(k for k in sd if k.startswith(prefix)):
        v = sd[k]
        if hasattr(v, "detach"):
            v = v.detach().cpu().contiguous().numpy()
        a = np.ascontiguousarray(v)
        h.update(k.encode() + b"\0" + str(a.dtype).encode() + str(a.shape).encode())
        h.update(a.tobytes())
    key = (h.hexdigest(), prefix, depth, act, tuple(sorted(kw.items())))
    hit = _PACK_CACHE.get(key)
    if hit is not None:
        _PACK_CACHE.move_to_end(key)
        return hit
    pb = pack_dense_block(sd, prefix, depth, act, **kw)
    _PACK_CACHE[key] = pb
    while len(_PACK_CACHE) > PACK_CACHE_MAX:
        _PACK_CACHE.popitem(last=False)
    return pb


def unpack_features(feat: np.ndarray, geom: BlockGeometry, n: int) -> np.ndarray:
    """Logical [P, n] view of the first n concatenated channels of a padded feature buffer."""
    return feat[:, geom.positions(n)]

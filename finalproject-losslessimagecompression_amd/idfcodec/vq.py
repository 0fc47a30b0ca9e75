"""The VQ-VAE of the residual configs on the device (vqvae.py:22-168; configs 3-5).

Every convolution is one `idf_conv_taps_f32` launch over a tap table (csrc/vq_kernels.hip):
Conv2d(k, s, p) is Hc = Ho, isy = s, taps (ky - p, kx - p); ConvTranspose2d(4, 2, 1) is four
launches, one per output parity (py, px), each a 2x2-tap conv on the input grid.  The 3x3
stride-1 convs (ResBlocks: 80-85% of the VQ-VAE's FLOPs) run as Winograd F(2x2, 3x3) instead,
residual add fused before the activation: by default as split-f16 products on f16 MFMA
(`idf_conv3x3_wx3_res`, conv mode "x3", the flow's own conv arithmetic, 1e-5 of fp32) with the
range guard -- a pass whose guard trips is recomputed with the exact-f32 Winograd kernel
(`idf_conv3x3_wino_res`, mode "f32").  The decoder's mode is part of the bitstream
(ResidualBitstream.vq_conv): the receiver rebuilds the same reconstruction.  Activations
are pixel-major with channel pitch round_up(C, 4); the 3-channel image is padded to 4 with
zeros (zero weights).  The batch_norm=True variants (BatchNorm after the activation,
vqvae.py:31-35) are rejected: no north-star config uses them.

Weight packing (`pack_conv`, `pack_convT`) is pure numpy, so it is testable without a GPU.

The quantiser and the reconstruction follow trainer.py:604-608: rec = round8(decoder(
embed[argmin]) * 0.5 + 0.5).  The decoder always runs on embed[idx] -- the value the
receiver can rebuild from the indices -- where the reference's straight-through
`x + (vq_x - x).detach()` (roundlib.py:66) can differ from embed[idx] by an ulp; the codec
is lossless either way because both sides run this same function.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr
from .packing import round_up

LEAKY = 0.01  # nn.LeakyReLU() default negative_slope


def _n_alloc(n: int) -> int:
    bn = 32 if n <= 32 else (64 if n <= 64 else 128)
    return round_up(n, bn)


@dataclass
class TapConv:
    """One packed conv launch: W [n_alloc][ntaps][ldw] (zero-padded)."""
    cin: int
    cout: int
    dy: list
    dx: list
    isy: int
    w: np.ndarray
    bias: np.ndarray
    osy: int = 1
    oy0: int = 0
    ox0: int = 0

    @property
    def ldw(self) -> int:
        return round_up(round_up(self.cin, 4), 16)

    @property
    def n_alloc(self) -> int:
        return self.w.shape[0]


def pack_conv(weight, bias, stride: int = 1, padding: int = 0) -> TapConv:
    """nn.Conv2d weight [co][ci][kh][kw] -> TapConv (taps row-major over (ky, kx))."""
    w = np.asarray(weight, np.float64)
    co, ci, kh, kw = w.shape
    b = np.zeros(co) if bias is None else np.asarray(bias, np.float64)
    dy = [ky - padding for ky in range(kh) for kx in range(kw)]
    dx = [kx - padding for ky in range(kh) for kx in range(kw)]
    ldw = round_up(round_up(ci, 4), 16)
    na = _n_alloc(co)
    wp = np.zeros((na, kh * kw, ldw), np.float32)
    wp[:co, :, :ci] = w.reshape(co, ci, kh * kw).transpose(0, 2, 1)
    bp = np.zeros(na, np.float32)
    bp[:co] = b
    return TapConv(ci, co, dy, dx, stride, wp, bp)


def pack_convT(weight, bias) -> list[TapConv]:
    """nn.ConvTranspose2d(k=4, s=2, p=1) weight [ci][co][4][4] -> four parity-class convs.
    Output row o = 2m + py receives input row i with o = 2i - 1 + ky, i.e. i = m + dy with
    (ky, dy) = (1, 0), (3, -1) for py = 0 and (0, +1), (2, 0) for py = 1 (same for x)."""
    w = np.asarray(weight, np.float64)
    ci, co, kh, kw = w.shape
    assert (kh, kw) == (4, 4)
    b = np.zeros(co) if bias is None else np.asarray(bias, np.float64)
    par = {0: [(1, 0), (3, -1)], 1: [(0, 1), (2, 0)]}
    ldw = round_up(round_up(ci, 4), 16)
    na = _n_alloc(co)
    out = []
    for py in (0, 1):
        for px in (0, 1):
            taps = [(ky, dy, kx, dx) for ky, dy in par[py] for kx, dx in par[px]]
            wp = np.zeros((na, 4, ldw), np.float32)
            for t, (ky, _, kx, _) in enumerate(taps):
                wp[:co, t, :ci] = w[:, :, ky, kx].T
            bp = np.zeros(na, np.float32)
            bp[:co] = b
            out.append(TapConv(ci, co, [t[1] for t in taps], [t[3] for t in taps], 1, wp, bp,
                               osy=2, oy0=py, ox0=px))
    return out


def taps_weights_x3(w: np.ndarray):
    """Split-f16 form of a TapConv's W [n_alloc][ntaps][ldw] for idf_conv_taps_x3: W * 2^k (k:
    packing.x3_scale, max |W| 2^k in [2^14, 2^15)) split wh = f16(w'), wl = f16(w' - wh) (both
    round-to-nearest-even, from the fp32 weights widened to float64), laid out per 4 channels as
    (wh[4], wl[4]) -- [n_alloc][ntaps][ldw / 4][8] uint16, the bytes of the fp32 array.  Returns
    (that array, yscale = 2^-k)."""
    from .packing import x3_scale
    w64 = np.asarray(w, np.float64)
    k = x3_scale(w64)
    ws = w64 * (2.0 ** k)
    hi = ws.astype(np.float16)
    lo = (ws - hi.astype(np.float64)).astype(np.float16)
    na, nt, ldw = w64.shape
    out = np.empty((na, nt, ldw // 4, 8), np.uint16)
    out[..., :4] = hi.view(np.uint16).reshape(na, nt, ldw // 4, 4)
    out[..., 4:] = lo.view(np.uint16).reshape(na, nt, ldw // 4, 4)
    return np.ascontiguousarray(out), float(2.0 ** -k)


def _np(t):
    return t.detach().cpu().double().numpy()


@dataclass
class Stage:
    """A conv launch in the network: kind 'conv' | 'convT' | 'res' (ResBlock = 2 convs)."""
    kind: str
    convs: list
    act: int           # IDF_ACT_* applied after the (last) conv
    stride: int = 1


def _seq_conv(seq):
    """nn.Sequential(Conv2d|ConvTranspose2d, act[, BatchNorm2d]) -> Stage.
    The reference applies BatchNorm AFTER the activation (vqvae.py:31-35), so it cannot be
    folded into the conv; those variants are rejected (no north-star config uses them)."""
    from torch import nn
    mods = list(seq)
    conv = mods[0]
    if any(isinstance(m, nn.BatchNorm2d) for m in mods):
        raise NotImplementedError("VQ-VAE batch_norm=True (BatchNorm after the activation) is not "
                                  "supported; the north-star configs use batch_norm: False")
    act = _lib.ACT["None"]
    for m in mods[1:]:
        if isinstance(m, nn.LeakyReLU):
            act = _lib.ACT["LeakyReLU"]
        elif isinstance(m, nn.ReLU):
            act = _lib.ACT["ReLU"]
        elif isinstance(m, nn.Tanh):
            act = _lib.ACT["Tanh"]
    if isinstance(conv, nn.ConvTranspose2d):
        return Stage("convT", pack_convT(_np(conv.weight), _np(conv.bias)), act, 2)
    s, p = conv.stride[0], conv.padding[0]
    return Stage("conv", [pack_conv(_np(conv.weight), _np(conv.bias), s, p)], act, s)


def _res_stage(block):
    """ResBlock (nnblock.py:59-84): relu(x + conv2(relu(conv1(x))))."""
    from torch import nn
    mods = list(block.resblock)
    if any(isinstance(m, nn.BatchNorm2d) for m in mods):
        raise NotImplementedError("ResBlock batch_norm=True is not supported (configs use False)")
    c1, c2 = mods[0], mods[2]
    return Stage("res", [pack_conv(_np(c1.weight), _np(c1.bias), 1, 1),
                         pack_conv(_np(c2.weight), _np(c2.bias), 1, 1)], _lib.ACT["ReLU"])


def encoder_stages(enc) -> list[Stage]:
    """VQEncoder.blocks (vqvae.py:22-63) then its Tanh."""
    from torch import nn
    st = []
    for blk in enc.blocks:
        if isinstance(blk, nn.Sequential):
            st.append(_seq_conv(blk))
        elif isinstance(blk, nn.Conv2d):
            st.append(Stage("conv", [pack_conv(_np(blk.weight), _np(blk.bias), 1, 0)],
                            _lib.ACT["None"]))
        else:
            st.append(_res_stage(blk))
    st[-1].act = _lib.ACT["Tanh"]  # self.act = nn.Tanh() after the last 1x1 (vqvae.py:60-62)
    return st


def decoder_stages(dec) -> list[Stage]:
    """VQDecoder.blocks (vqvae.py:66-113)."""
    from torch import nn
    return [_seq_conv(b) if isinstance(b, nn.Sequential) else _res_stage(b) for b in dec.blocks]


def is_wino(c: TapConv) -> bool:
    """Conv2d(k=3, s=1, p=1) with channel counts the Winograd kernel takes."""
    return (len(c.dy) == 9 and c.isy == 1 and c.osy == 1 and c.cin % 4 == 0
            and list(zip(c.dy, c.dx)) == [(y, x) for y in (-1, 0, 1) for x in (-1, 0, 1)])


class DevConv:
    def __init__(self, c: TapConv, device, wino: bool = True):
        self.c = c
        self.w = torch.from_numpy(c.w).to(device)
        self.wino_u = self.wx3_u = None
        self.wx3_yscale = 1.0
        if wino and is_wino(c):
            from .packing import wino_transform64, wino_weights, wino_weights_x3
            nslab = c.ldw // 16
            U = wino_transform64(c.w.astype(np.float64), nslab)
            self.wino_u = torch.from_numpy(wino_weights(c.w.astype(np.float64), nslab, U)).to(device)
            ux3, self.wx3_yscale = wino_weights_x3(c.w.astype(np.float64), nslab, U)
            self.wx3_u = torch.from_numpy(ux3.view(np.int16)).to(device)
        # the tap GEMM's split-f16 weights (VQ conv mode "x3t", idf_conv_taps_x3)
        self.wt_x3 = None
        self.wt_yscale = 1.0
        if wino and self.wino_u is None:
            wt, self.wt_yscale = taps_weights_x3(c.w)
            self.wt_x3 = torch.from_numpy(wt.view(np.int16)).to(device)
        self.b = torch.from_numpy(c.bias).to(device)
        self.dy = (ctypes.c_int32 * len(c.dy))(*c.dy)
        self.dx = (ctypes.c_int32 * len(c.dx))(*c.dx)


# "x3t": ResBlock 3x3 convs on split-f16 Winograd (wx3) and every other conv on the split-f16
# tap GEMM (idf_conv_taps_x3); "x3": round 3-5's -- wx3 ResBlocks, the other convs in exact fp32;
# "f32": everything exact fp32.  The decoder runs the mode its bitstream records.
VQ_CONV_MODES = ("x3t", "x3", "f32")
SPLIT_VQ = ("x3t", "x3")


class VQEngine:
    """Device VQ-VAE: indices and reconstruction of a batch of images.

    conv_mode ("x3t" default, IDF_VQ_CONV overrides; VQ_CONV_MODES): the arithmetic of the convs.
    argmin_mode ("x3" default, IDF_VQ_ARGMIN overrides; "f32"): the codebook search's x.e products
    (split-f16 MFMA, fp32-class, or fp32 MFMA).  Encoder-side only -- the decoder reads the
    indices from the stream -- so it is not recorded.
    encode_pm / decode_pm run it and fall back to "f32" for the whole pass when the split-f16
    range guard trips; last_decode_mode is the mode the last decode_pm ran (what the encoder
    records for its receiver)."""

    def __init__(self, model, device, wino: bool = True):
        import os
        self.device = device
        self.wino = wino
        self.conv_mode = os.environ.get("IDF_VQ_CONV", "x3t") if wino else "f32"
        if self.conv_mode not in VQ_CONV_MODES:
            raise ValueError(f"IDF_VQ_CONV={self.conv_mode!r}: one of {VQ_CONV_MODES}")
        self.last_decode_mode = self.conv_mode
        self.argmin_mode = os.environ.get("IDF_VQ_ARGMIN", "x3") if wino else "f32"
        if self.argmin_mode not in ("x3", "f32"):
            raise ValueError(f"IDF_VQ_ARGMIN={self.argmin_mode!r}: 'x3' or 'f32'")
        # bench timing (tools/bench_residual.py vq_roofline): when a list, every conv and argmin
        # launch appends (kind, algorithmic FLOPs, event before, event after) on its stream
        self.timer = None
        self.flag = torch.zeros(1, dtype=torch.int32, device=device)
        self._mode = self.conv_mode  # the mode of the pass being run
        self._ws = None
        self.channel = model.channel
        self.D = model.embed_dim
        self.K = model.embed_num
        self.enc = [self._dev(s) for s in encoder_stages(model.encoder)]
        self.dec = [self._dev(s) for s in decoder_stages(model.decoder)]
        self.embed = model.vq.embed.weight.detach().float().contiguous().to(device)
        self.enorm = torch.empty(self.K, dtype=torch.float32, device=device)
        check(lib().idf_vq_norms(_lib.stream_ptr(device), self.K, self.D, ptr(self.embed), self.D,
                                 ptr(self.enorm)), "vq norms")
        self.embed_x3 = None
        if self.D % 4 == 0:  # split codebook for idf_vq_argmin_x3_ws
            ex, self.embed_yscale = taps_weights_x3(_np(model.vq.embed.weight).reshape(
                self.K, 1, self.D))
            self.embed_x3 = torch.from_numpy(ex.reshape(-1)).to(device)

    def _dev(self, st: Stage):
        return (st, [DevConv(c, self.device, self.wino) for c in st.convs])

    # ---------------------------------------------------------------- conv runner
    def _timed(self, kind, flops):
        """(start, finish) callables around one launch: HIP events on the current stream when
        self.timer is a list, no-ops otherwise."""
        if self.timer is None:
            return lambda: None, lambda: None
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        self.timer.append((kind, float(flops), a, b))
        return a.record, b.record

    def _conv(self, s, dc: DevConv, x, B, H, W, ldx, act, out, ldo, Ho, Wo, res=None, ldr=0,
              check_in=1):
        c = dc.c
        if self.timer is not None:
            # algorithmic FLOPs: 2 x taps x cin x cout per computed output (the Winograd 3x3
            # priced as the direct conv it computes; a transposed conv's launch covers one output
            # parity: its taps on the input grid)
            grid = B * (H * W if (dc.wino_u is not None or c.osy == 2) else Ho * Wo)
            split = self._mode in SPLIT_VQ
            kind = (("resblock3x3_x3" if split else "resblock3x3_f32") if dc.wino_u is not None
                    else ("conv_taps_x3" if self._mode == "x3t" and dc.wt_x3 is not None
                          else "conv_taps"))
            t0, t1 = self._timed(kind, 2.0 * grid * len(c.dy) * c.cin * c.cout)
        else:
            t0 = t1 = lambda: None
        t0()
        self._conv_launch(s, dc, x, B, H, W, ldx, act, out, ldo, Ho, Wo, res, ldr, check_in)
        t1()

    def _conv_launch(self, s, dc: DevConv, x, B, H, W, ldx, act, out, ldo, Ho, Wo, res, ldr,
                     check_in):
        c = dc.c
        if dc.wino_u is not None:
            L = lib()
            wsn = int(L.idf_conv3x3_wino_workspace(B, H, W, c.cin, c.cout))
            ws = self._wino_ws(wsn)
            if self._mode in SPLIT_VQ:
                check(L.idf_conv3x3_wx3_res(
                    s, B, H, W, c.cin, ptr(x), ldx, ptr(dc.wx3_u), c.n_alloc // 16,
                    dc.wx3_yscale, ptr(dc.b), c.cout, ptr(out), ldo,
                    ptr(res) if res is not None else None, ldr, act, LEAKY, ptr(self.flag),
                    check_in, ptr(ws) if wsn else None, wsn), "vq wx3 conv")
                return
            check(L.idf_conv3x3_wino_res(
                s, B, H, W, c.cin, ptr(x), ldx, ptr(dc.wino_u), c.n_alloc // 16, ptr(dc.b), c.cout,
                ptr(out), ldo, ptr(res) if res is not None else None, ldr, act, LEAKY,
                ptr(ws) if wsn else None, wsn), "vq wino conv")
            return
        if c.osy == 2:      # transposed: compute grid = input grid
            Hc, Wc = H, W
        else:
            Hc, Wc = Ho, Wo
        if self._mode == "x3t" and dc.wt_x3 is not None:
            check(lib().idf_conv_taps_x3(
                s, B, H, W, round_up(c.cin, 4), ptr(x), ldx, Hc, Wc, c.isy, c.isy, len(c.dy), dc.dy,
                dc.dx, ptr(dc.wt_x3), c.ldw, c.n_alloc, dc.wt_yscale, ptr(dc.b), c.cout, ptr(out),
                ldo, Ho, Wo, c.osy, c.osy, c.oy0, c.ox0, ptr(res) if res is not None else None, ldr,
                act, LEAKY, ptr(self.flag)), "vq conv x3t")
            return
        check(lib().idf_conv_taps_f32(
            s, B, H, W, round_up(c.cin, 4), ptr(x), ldx, Hc, Wc, c.isy, c.isy, len(c.dy), dc.dy,
            dc.dx, ptr(dc.w), c.ldw, c.n_alloc, ptr(dc.b), c.cout, ptr(out), ldo, Ho, Wo, c.osy,
            c.osy, c.oy0, c.ox0, ptr(res) if res is not None else None, ldr, act, LEAKY),
            "vq conv")

    def _wino_ws(self, n):
        if n and (self._ws is None or self._ws.numel() < n):
            self._ws = torch.empty(n, dtype=torch.float32, device=self.device)
        return self._ws

    def _guarded(self, stages, x, B, H, W, C, mode=None):
        """_run in `mode` (default conv_mode); an "x3" pass whose range guard trips is run
        again in "f32".  Returns (outputs..., the mode that produced them)."""
        mode = mode or self.conv_mode
        if mode not in VQ_CONV_MODES:
            raise ValueError(f"unknown VQ conv mode {mode!r}")
        if mode in SPLIT_VQ:
            self.flag.zero_()
        self._mode = mode
        out = self._run(stages, x, B, H, W, C)
        if mode in SPLIT_VQ and bool(self.flag.item()):
            self._mode = mode = "f32"
            out = self._run(stages, x, B, H, W, C)
        self._mode = self.conv_mode
        return out + (mode,)

    def _run(self, stages, x, B, H, W, C):
        """Run conv stages on a pixel-major buffer x [B*H*W][round_up(C,4)]."""
        s = _lib.stream_ptr(self.device)
        for st, dcs in stages:
            ldx = round_up(C, 4)
            if st.kind == "conv":
                c = dcs[0].c
                Ho, Wo = H // c.isy if c.isy > 1 else H, W // c.isy if c.isy > 1 else W
                ldo = round_up(c.cout, 4)
                y = torch.empty(B * Ho * Wo * ldo, dtype=torch.float32, device=self.device)
                if ldo != c.cout:
                    y.zero_()
                self._conv(s, dcs[0], x, B, H, W, ldx, st.act, y, ldo, Ho, Wo)
                x, H, W, C = y, Ho, Wo, c.cout
            elif st.kind == "convT":
                c = dcs[0].c
                Ho, Wo = 2 * H, 2 * W
                ldo = round_up(c.cout, 4)
                y = torch.empty(B * Ho * Wo * ldo, dtype=torch.float32, device=self.device)
                if ldo != c.cout:
                    y.zero_()
                for dc in dcs:
                    self._conv(s, dc, x, B, H, W, ldx, st.act, y, ldo, Ho, Wo)
                x, H, W, C = y, Ho, Wo, c.cout
            else:  # ResBlock: t = relu(conv1(x)); x = relu(x + conv2(t))
                t = torch.empty_like(x)
                self._conv(s, dcs[0], x, B, H, W, ldx, _lib.ACT["ReLU"], t, ldx, H, W)
                y = torch.empty_like(x)
                # t is a guarded conv output (|t| < 8192): its transform needs no input check
                self._conv(s, dcs[1], t, B, H, W, ldx, st.act, y, ldx, H, W, res=x, ldr=ldx,
                           check_in=0)
                x = y
        return x, H, W, C

    # ---------------------------------------------------------------- API
    def encode_pm(self, data_pm, B, H, W):
        """data on the 1/256 grid, pixel-major [B*H*W][4] (channels padded to 4) ->
        int32 indices [B * H/d * W/d] (trainer.py:606 input scaling, vqvae.py:135-147)."""
        s = _lib.stream_ptr(self.device)
        P = B * H * W
        x = torch.zeros(P * 4, dtype=torch.float32, device=self.device)
        check(lib().idf_vq_pointwise(s, P, self.channel, 0, ptr(data_pm), 4, None, 0, ptr(x), 4),
              "vq scale in")
        z, h, w, C, _ = self._guarded(self.enc, x, B, H, W, self.channel)
        assert C == self.D
        idx = torch.empty(B * h * w, dtype=torch.int32, device=self.device)
        nws = int(lib().idf_vq_argmin_workspace_bytes(B * h * w, self.K))
        ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=self.device)
        split = self.argmin_mode == "x3" and self.embed_x3 is not None
        if split:
            self.flag.zero_()
        t0, t1 = self._timed("argmin_x3" if split else "argmin", 2.0 * B * h * w * self.D * self.K)
        def fp32():
            check(lib().idf_vq_argmin_ws(s, B * h * w, self.D, ptr(z), round_up(self.D, 4),
                                         ptr(self.embed), self.D, self.K, ptr(self.enorm),
                                         ptr(idx), ptr(ws), nws), "vq argmin")
        t0()
        if split:
            check(lib().idf_vq_argmin_x3_ws(s, B * h * w, self.D, ptr(z), round_up(self.D, 4),
                                            ptr(self.embed_x3), self.D, self.embed_yscale, self.K,
                                            ptr(self.enorm), ptr(idx), ptr(ws), nws,
                                            ptr(self.flag)), "vq argmin x3")
        else:
            fp32()
        t1()
        if split and bool(self.flag.item()):  # the range guard: search again in fp32
            fp32()
        return idx, (h, w), z

    def decode_pm(self, idx, B, h, w, mode=None):
        """indices -> rec on the 1/256 grid, pixel-major [B*H*W][4] (vqvae.py:149-151,
        trainer.py:606-607: rec = round8(decoder(embed[idx]) * 0.5 + 0.5)).  mode: the conv
        arithmetic to reproduce (a decoder passes the bitstream's vq_conv); default conv_mode
        with the guard's fallback.  The mode that ran is left in last_decode_mode."""
        s = _lib.stream_ptr(self.device)
        P = B * h * w
        D4 = round_up(self.D, 4)
        v = torch.zeros(P * D4, dtype=torch.float32, device=self.device)
        check(lib().idf_vq_gather(s, P, self.D, ptr(idx), ptr(self.embed), self.D, ptr(v), D4),
              "vq gather")
        y, H, W, C, self.last_decode_mode = self._guarded(self.dec, v, B, h, w, self.D, mode)
        assert C == self.channel
        rec = torch.zeros(B * H * W * 4, dtype=torch.float32, device=self.device)
        check(lib().idf_vq_pointwise(s, B * H * W, C, 1, ptr(y), 4, None, 0, ptr(rec), 4),
              "vq rec")
        return rec, (H, W)

    def decoder_raw_pm(self, vq_pm, B, h, w):
        """decoder output (tanh range, pixel-major, pitch 4) for a given latent (tests)."""
        y, H, W, C, _ = self._guarded(self.dec, vq_pm, B, h, w, self.D)
        return y, (H, W)

    def encoder_raw_pm(self, x_pm, B, H, W):
        """encoder output (tanh, pixel-major pitch round_up(D,4)) for a scaled input (tests)."""
        z, h, w, C, _ = self._guarded(self.enc, x_pm, B, H, W, self.channel)
        return z, (h, w)

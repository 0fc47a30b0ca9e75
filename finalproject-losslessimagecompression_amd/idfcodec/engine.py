"""FlowEngine: the IDF forward (encode side) and inverse (decode side) on the GPU.

Runs the reference hot path (flows.py:87-152, couplelib.py:47-61,
priorlib.py:36-47, nnblock.py:53-56, invertible.py:38-48, extenddim.py:23-37)
entirely through libidfcodec.so kernels.  torch only provides device memory
and the stream.

HBM layout (per batch of B images):
  x_l   : two pixel-major buffers per level [B*h_l*w_l, ldx_l] (ping-pong across
          couplings; the permutation is a gather between them)
  feat  : DenseBlock feature buffer [P, ld_feat] shared by all blocks
  tmp   : 1x1-conv output [P, ld_feat]
  lat / mean / logscale / scale : flat f32 [B * n_sym], level-major, image-minor,
          NCHW inside -- so rANS stream (image b, level l) is one contiguous run
          in the reference's symbol order (x[i].reshape(-1), trainer.py:311).
"""
from __future__ import annotations

import collections
import ctypes
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import IdfDenseBlock, IdfError, IdfHeadOut, check, lib, ptr
from .packing import PackedBlock, pack_dense_block_cached, round_up

FLOAT = 4
CONV_MODES = ("dx3", "dx3w16", "x3", "f32")
# the split-f16 modes (the range guard applies; fallback: exact-f32 "f32")
SPLIT_F16 = ("dx3", "dx3w16", "x3")
# Fold each DenseLayer's 1x1 conv into its 3x3 conv (packing.fold_layer): -46% of the
# flow FLOPs at imagenet64; IDF_FOLD=0 runs the reference's two convolutions instead.
FOLD = os.environ.get("IDF_FOLD", "1") != "0"
# Folded 3x3 convs run on the LDS halo-tiled kernel (conv3_halo.hip); IDF_HALO=0 selects
# the implicit-GEMM kernel instead (A/B comparisons).
HALO = os.environ.get("IDF_HALO", "1") != "0"
# Folded 3x3 convs on even-sized images run as Winograd F(2x2,3x3) (conv3_wino.hip, 2.25x
# fewer multiplies); IDF_WINO=0 keeps them on the direct halo kernel.
WINO = os.environ.get("IDF_WINO", "1") != "0"
# fp32 Winograd convs use split-f16 products (idf_conv3x3_wx3: each f32 operand as an f16
# hi/lo pair, three f16 MFMAs, f32 accumulation -- fp32-class error) with a
# range guard that falls back to the exact-f32 kernel; IDF_WX3=0 always uses the latter.
WX3 = os.environ.get("IDF_WX3", "1") != "0"
# ... and, where the geometry allows (conv3_dx3.hip dx3_plan: widths a multiple of 16, packed
# 8- and 4-wide images, bands of wider ones), as the direct conv on the same split-f16 products
# with no transform ("dx3", the default mode); IDF_DX3=0 keeps every layer on wx3.  Conv modes:
# 'dx3' (dx3 where supported, wx3 elsewhere), 'dx3w16' (round 4's dx3: only widths a multiple of
# 16 on dx3 -- decodes version-2 files with conv code 6), 'x3', 'f32'; the mode is recorded in
# the bitstream.
DX3 = os.environ.get("IDF_DX3", "1") != "0"
# In 'dx3' mode a DenseBlock whose layers all run on dx3 (one output group) with a head of <= 16
# outputs (every coupling, the 32x32 prior) fuses the head into its layers: running sums from
# the block input (idf_dx3_head_init), each layer's epilogue adds its outputs' share, the last
# applies the coupling / prior epilogue -- no head GEMM re-reading the feature buffer, and the
# layers skip their fp32 output stores (IdfDenseBlock.fuse_head / keep_feat).  The fusion is part
# of the conv arithmetic the mode names (the head's sums run in another order than the GEMM's):
# on in modes 'dx3' and 'dxb', off in 'dx3w16', decided by the block geometry alone -- no switch,
# so an encoder and its decoder cannot disagree on it.
# Blocks whose layers all run on dx3 / dxb at a geometry whose tiles hold whole images (the
# 16x16 and 8x8 levels, config 4's 4x4 patches) run as ONE launch per DenseBlock, a workgroup per
# tile looping over the layers (IdfDenseBlock.fuse_layers, conv3_dx3_block_kernel): bit for bit
# the per-layer launches' results, so not part of the bitstream; IDF_FUSE_LAYERS=0 keeps one
# launch per layer (A/B timing, the equivalence tests).
# IDF_FUSE_LAYERS: "1" every level the kernel takes, "0" none, or a comma list of level heights
# (e.g. "8,4").
_FL = os.environ.get("IDF_FUSE_LAYERS", "1")
FUSE_LAYERS = _FL != "0"
FUSE_LEVELS = None if _FL in ("0", "1") else {int(v) for v in _FL.split(",") if v}
# bf16 engines (configs naming bf16 coupling convs) run their DenseLayers as the bf16 direct
# conv (conv mode "dxb", idf_conv3x3_dxb: the dx3 kernel's tiling and LDS-DMA with one bf16
# product per tap) where the level geometry allows, conv3_bf16.hip ("bf16", round 4's) elsewhere
# and when IDF_DXB=0.  The two sum in different orders: a bitstream records which ran.
DXB = os.environ.get("IDF_DXB", "1") != "0"
BF16_MODES = ("dxb", "bf16")


class DeviceBlock:
    """A packed DenseBlock resident in HBM plus its C descriptor."""

    def __init__(self, packed: PackedBlock, device):
        self.packed = packed
        self.geom = packed.geom
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        self.w1 = [dev(a) for a in packed.w1]
        self.b1 = [dev(a) for a in packed.b1]
        self.w3 = [dev(a) for a in packed.w3]
        self.b3 = [dev(a) for a in packed.b3]
        self.wh = dev(packed.wh)
        self.bh = dev(packed.bh)
        self.vtap = [dev(a) for a in packed.vtap]
        self.bfull = [dev(a) for a in packed.bfull]
        self.wino_u = [dev(a) for a in packed.wino_u]
        self.wb16 = [dev(a.view(np.int16)) for a in packed.wb16]
        self.wx3_u = [dev(a.view(np.int16)) for a in packed.wx3_u]
        self.dx3_w = [dev(a.view(np.int16)) for a in packed.dx3_w]
        self.dxb_w = [dev(a.view(np.int16)) for a in packed.dxb_w]
        d = IdfDenseBlock()
        g = self.geom
        d.depth = g.depth
        d.act = _lib.ACT[packed.act]
        d.slope = packed.slope
        d.g_pad = g.g_pad
        d.g_alloc = packed.g_alloc
        for i, k in enumerate(g.k_in):
            d.k_in[i] = k
        for i in range(g.depth):
            d.n1_alloc[i] = packed.n1_alloc[i]
            d.ldw1[i] = packed.ldw1[i]
            d.ldw3[i] = packed.ldw3[i]
            d.w1[i] = self.w1[i].data_ptr()
            d.b1[i] = self.b1[i].data_ptr()
            d.w3[i] = self.w3[i].data_ptr()
            d.b3[i] = self.b3[i].data_ptr()
        d.n_head = g.n_head
        d.nh_alloc = packed.nh_alloc
        d.ldwh = packed.ldwh
        d.wh = self.wh.data_ptr()
        d.bh = self.bh.data_ptr()
        c = g.a
        for i in range(g.depth):
            d.c_real[i] = c
            d.g_real[i] = g.growth[i]
            c += g.growth[i]
        d.c_real[g.depth] = c
        d.fold = 1 if packed.fold else 0
        d.halo = 1 if (packed.fold and HALO) else 0
        d.wino = 1 if (packed.fold and self.wino_u) else 0
        d.wino_nft = packed.g_alloc // 16
        for i, u in enumerate(self.wino_u):
            d.wino_u[i] = u.data_ptr()
        d.wx3 = 1 if (d.wino and self.wx3_u) else 0
        for i, u in enumerate(self.wx3_u):
            d.wx3_u[i] = u.data_ptr()
            d.wx3_yscale[i] = packed.wx3_yscale[i]
        d.dx3 = 1 if (d.wx3 and self.dx3_w) else 0
        d.fuse_head = 1 if d.dx3 else 0
        d.keep_feat = 0
        for i, w in enumerate(self.dx3_w):
            d.dx3_w[i] = w.data_ptr()
            d.dx3_yscale[i] = packed.dx3_yscale[i]
        d.bf16 = 1 if (packed.fold and self.wb16) else 0
        for i, u in enumerate(self.wb16):
            d.wb16[i] = u.data_ptr()
        d.dxb = 1 if (d.bf16 and self.dxb_w and DXB) else 0
        d.fuse_head = 1 if (d.dx3 or d.dxb) else 0
        d.fuse_layers = 1 if FUSE_LAYERS else 0
        for i, u in enumerate(self.dxb_w):
            d.dxb_w[i] = u.data_ptr()
        d.ldv = packed.g_alloc
        for i in range(len(self.vtap)):
            d.vtap[i] = self.vtap[i].data_ptr()
            d.bfull[i] = self.bfull[i].data_ptr()
        self.desc = d
        self.timer = None  # an IdfTimer handle: when set, GEMM launches are event-timed

    def run(self, stream, B, H, W, feat, ld_feat, tmp, ld_tmp, head: IdfHeadOut | None):
        h = ctypes.byref(head) if head else None
        if self.timer is not None:
            check(lib().idf_dense_block_f32_timed(stream, ctypes.byref(self.desc), B, H, W, feat,
                                                  ld_feat, tmp, ld_tmp, h, self.timer),
                  "idf_dense_block_f32_timed")
        else:
            check(lib().idf_dense_block_f32(stream, ctypes.byref(self.desc), B, H, W, feat, ld_feat,
                                            tmp, ld_tmp, h), "idf_dense_block_f32")


def head_couple(mode, out_ptr, ld):
    h = IdfHeadOut()
    h.mode = mode
    h.out = out_ptr
    h.ld_out = ld
    h.base = out_ptr
    h.ld_base = ld
    return h


def head_prior(n_mean, mean_ptr, logscale_ptr, scale_ptr):
    h = IdfHeadOut()
    h.mode = _lib.EPI_PRIOR
    h.n_mean = n_mean
    h.mean = mean_ptr
    h.logscale = logscale_ptr
    h.scale = scale_ptr
    return h


@dataclass
class Level:
    C: int          # channels after squeeze
    h: int
    w: int
    a: int          # coupling a_ch (couplelib.py:38)
    z: int          # latent channels
    rest: int       # channels passed on (C - z)
    ldx: int
    cond_ch: int    # ConditionalFlows cond channels at this level (0 for IDFlows)
    prior_x_zero: bool  # prior sees zeros for the x part (top level)

    @property
    def n_sym(self) -> int:
        return self.z * self.h * self.w


class FlowEngine:
    """Built from a model exposing the reference attributes/state_dict
    (IDFlows / ConditionalFlows of this package)."""

    def __init__(self, model, device=None, fold: bool | None = None):
        self.device = torch.device(device or "cuda")
        # "bf16": the DenseLayer convs run on bf16 MFMA (configs naming bf16 coupling convs,
        # e.g. resflow-cond-imagenet64); "f32" (default): fp32, within 1e-5 of the reference
        self.precision = getattr(model, "idf_precision", "f32")
        if self.precision not in ("f32", "bf16"):
            raise ValueError(f"idf_precision must be 'f32' or 'bf16', not {self.precision!r}")
        self.fold = FOLD if fold is None else bool(fold)
        if self.precision == "bf16":
            self.fold = True
        self.wino = self.fold and WINO and self.precision == "f32" and any(
            lib().idf_conv3x3_wino_supported(model.H // s, model.W // s)
            for s in [model.blocks[0]["extend"].scale ** (l + 1) for l in range(model.nsplit)])
        self.wx3 = self.wino and WX3
        self.dx3 = self.wx3 and DX3 and any(
            lib().idf_conv3x3_dx3_supported(model.H // s, model.W // s, 48)
            for s in [model.blocks[0]["extend"].scale ** (l + 1) for l in range(model.nsplit)])
        # device word the wx3 range guard ORs into (see IdfDenseBlock.range_flag)
        self.range_flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        sd = {k: v for k, v in model.state_dict().items()}
        self.conditional = type(model).__name__ == "ConditionalFlows"
        self.conv_for_cond = bool(getattr(model, "conv_for_cond", False))
        self.nflows = model.nflows
        self.nsplit = model.nsplit
        self.C, self.H, self.W = model.C, model.H, model.W
        self.scale = model.blocks[0]["extend"].scale
        split = model.blocks[0]["flows"][1].split
        c_depth = model.blocks[0]["flows"][1].dense.depth
        c_act = model.blocks[0]["flows"][1].dense.act_name
        p_depth = model.blocks[0]["prior"].NN.depth
        p_act = model.blocks[0]["prior"].NN.act_name
        self.levels: list[Level] = []
        ch, h, w = self.C, self.H, self.W
        cond_ch = self.C
        for l in range(self.nsplit):
            ch *= self.scale * self.scale
            h //= self.scale
            w //= self.scale
            cond_ch *= self.scale * self.scale
            top = l == self.nsplit - 1
            z = ch if top else ch // 2
            self.levels.append(Level(C=ch, h=h, w=w, a=int(ch * split), z=z, rest=ch - z,
                                     ldx=round_up(ch, 4),
                                     cond_ch=cond_ch if self.conditional else 0,
                                     prior_x_zero=top))
            if not top:
                ch -= ch // 2
        self.n_sym_img = sum(L.n_sym for L in self.levels)
        # device weights
        self.couple = []
        self.prior = []
        self.ids = []
        self.inv_ids = []
        for l in range(self.nsplit):
            self.couple.append([DeviceBlock(pack_dense_block_cached(
                sd, f"blocks.{l}.flows.{2 * k + 1}.dense.", c_depth, c_act, fold=self.fold,
                wino=self.wino, bf16=self.precision == "bf16", wx3=self.wx3,
                dx3=self.dx3 and self._dx3_level(l), dx3_cmax=self._dx3_cmax(l)),
                self.device) for k in range(self.nflows)])
            self.prior.append(DeviceBlock(pack_dense_block_cached(sd, f"blocks.{l}.prior.NN.", p_depth,
                                                           p_act, fold=self.fold, wino=self.wino,
                                                           bf16=self.precision == "bf16",
                                                           wx3=self.wx3,
                                                           dx3=self.dx3 and self._dx3_level(l),
                                                           dx3_cmax=self._dx3_cmax(l)),
                                          self.device))
            ids_l, inv_l = [], []
            for k in range(self.nflows + 1):
                Pm = sd[f"blocks.{l}.flows.{2 * k}.P"].detach().float().cpu()
                ids = torch.argmax(Pm, dim=1).to(torch.int32)
                inv = torch.empty_like(ids)
                inv[ids.long()] = torch.arange(ids.numel(), dtype=torch.int32)
                ids_l.append(ids.to(self.device))
                inv_l.append(inv.to(self.device))
            self.ids.append(ids_l)
            self.inv_ids.append(inv_l)
        if self.conv_for_cond:
            # Conv2d(c, 4c, 4, 2, 1) (flows.py:298-301) as an implicit GEMM on the MFMA tap
            # kernel shared with the VQ-VAE (vq_kernels.hip conv_taps_kernel)
            from .vq import DevConv, pack_conv
            self.cond_conv = [DevConv(pack_conv(sd[f"convs.{l}.weight"].detach().double().cpu(),
                                                sd[f"convs.{l}.bias"].detach().double().cpu(),
                                                stride=2, padding=1), self.device)
                              for l in range(self.nsplit)]
        blocks = [b for lv in self.couple for b in lv] + self.prior
        self._blocks = blocks
        for b in blocks:
            b.desc.range_flag = self.range_flag.data_ptr()
        if FUSE_LEVELS is not None:
            for l, L in enumerate(self.levels):
                for b in self.couple[l] + [self.prior[l]]:
                    b.desc.fuse_layers = 1 if L.h in FUSE_LEVELS else 0
        self.conv_mode = "dx3" if self.dx3 else ("x3" if self.wx3 else "f32")
        self.dxb = self.precision == "bf16" and DXB and any(b.dxb_w for b in blocks)
        if self.precision == "bf16":
            self.conv_mode = "dxb" if self.dxb else "bf16"
        self.ld_feat = max(b.geom.ld_feat for b in blocks)
        # tmp: split-K partials (f32); bf16 blocks also keep their bf16 feature shadow at its
        # front (pitch round_up(k, 64) bf16 = half as many floats) ahead of 2-way partials
        self.ld_tmp = self.ld_feat
        if self.precision == "bf16":
            self.ld_tmp = max(self.ld_feat, round_up(self.ld_feat, 64) // 2 + 2 * 48 + 8)
        self._ws = collections.OrderedDict()
        self.ws_keep = 4
        # IDFlows' data-independent top prior, one entry per conv mode, never dropped: an
        # encode on one stream may switch the mode (the range guard's f32 recompute) while a
        # decode on another still has copies from the current mode's entry queued
        self._top_prior = {}

    # ------------------------------------------------------------ conv mode
    def _dx3_level(self, l: int) -> bool:
        Lv = self.levels[l]
        return bool(lib().idf_conv3x3_dx3_supported(Lv.h, Lv.w, 48))

    def _dx3_cmax(self, l: int):
        """Widest (16-padded) layer input level l runs on dx3 (None: every layer); wider layers
        of a block run on wx3.  A function of the level geometry only, never of the batch, so
        an encoder and a decoder of the same model pick the same arithmetic for every layer.
        Every layer: the same-box bench A/B (profiles/r04/dx3_prefix/bench_ab.txt) measured
        all-dx3 19.18/19.08 Mpx/s against 18.59/18.76 for dx3 up to 232/152 input channels at
        32x32/16x16 and 18.41/18.50 for none, although the isolated-launch sweep there has wx3
        ahead from ~188 channels."""
        return None

    def _dx3_level_in(self, l: int, mode: str) -> bool:
        """Level l's DenseLayers run on dx3 under conv mode `mode`."""
        return mode in ("dx3", "dx3w16") and self._dx3_level(l) and (
            mode == "dx3" or self.levels[l].w % 16 == 0)

    def dx3_layers(self, l: int, geom) -> int:
        """Leading layers of a level-l block with geometry `geom` that run on dx3."""
        if not self._dx3_level_in(l, self.conv_mode):
            return 0
        cm = self._dx3_cmax(l)
        return sum(1 for i in range(geom.depth) if cm is None or geom.k_in[i] <= cm)

    def fused_block(self, l: int, blk) -> bool:
        """Whether level l's block `blk` runs as one fused launch (IdfDenseBlock.fuse_layers):
        every layer on dx3 / dxb at a geometry whose tiles hold whole images."""
        d = blk.desc
        if not d.fuse_layers or not (d.dx3 or d.dxb):
            return False
        if d.dx3 and self.dx3_layers(l, blk.geom) != blk.geom.depth:
            return False
        L = self.levels[l]
        return bool(lib().idf_dx3_block_supported(L.h, L.w, blk.geom.g_pad, 1 if d.dxb else 0))

    def set_conv_mode(self, mode: str):
        """'dx3' (split-f16 direct conv where the geometry allows, split-f16 Winograd
        elsewhere), 'x3' (split-f16 Winograd everywhere; both need the split weights) or 'f32'
        (exact-f32 Winograd).  The decoder must run the mode the encoder ran
        (Bitstream.meta['conv'])."""
        if self.precision == "bf16":
            if mode not in BF16_MODES or (mode == "dxb" and not self.dxb):
                raise ValueError(f"this bf16 engine runs conv modes "
                                 f"{BF16_MODES if self.dxb else ('bf16',)}, not {mode!r}")
            for b in self._blocks:
                b.desc.dxb = 1 if (mode == "dxb" and b.dxb_w) else 0
                b.desc.fuse_head = 1 if b.desc.dxb else 0
            self.conv_mode = mode
            return
        if mode not in CONV_MODES:
            raise ValueError(f"conv mode must be one of {CONV_MODES}, not {mode!r}")
        if mode == "x3" and not self.wx3:
            raise ValueError("this engine has no split-f16 (wx3) weights")
        if mode in ("dx3", "dx3w16") and not self.dx3:
            raise ValueError("this engine has no split-f16 direct-conv (dx3) weights")
        on = 1 if mode in SPLIT_F16 else 0
        for l in range(self.nsplit):
            dl = self._dx3_level_in(l, mode)
            for b in self.couple[l] + [self.prior[l]]:
                b.desc.wx3 = on if b.wx3_u else 0
                b.desc.dx3 = 1 if (dl and b.dx3_w and b.desc.wx3) else 0
                # round 5's dx3 fuses the heads; dx3w16 (round 4's arithmetic) keeps the GEMMs
                b.desc.fuse_head = 1 if (mode == "dx3" and b.desc.dx3) else 0
        self.conv_mode = mode  # each mode's top prior is cached separately (_top_prior)

    @property
    def conv_family(self) -> str:
        """Which conv arithmetic produces the couplings -- the decoder must run the same one
        (Bitstream.meta['conv']): 'dx3' / 'dx3w16' / 'x3' / 'f32' (split-f16 direct + Winograd / split-f16
        Winograd / exact-f32 Winograd, switchable per bitstream), 'bf16', 'halo' (direct
        LDS-halo kernel), 'gemm' (folded implicit GEMM) or 'unfold' (the reference's 1x1 +
        3x3, IDF_FOLD=0)."""
        if self.precision == "bf16":
            return self.conv_mode  # "dxb" or "bf16"
        if not self.fold:
            return "unfold"
        if self.wino:
            return self.conv_mode
        return "halo" if HALO else "gemm"

    def can_run(self, conv: str) -> bool:
        """This engine can switch to conv mode `conv` (a bitstream's recorded arithmetic)."""
        if self.precision == "bf16":
            return conv == "bf16" or (conv == "dxb" and self.dxb)
        if not (self.fold and self.wino):
            return False
        return conv == "f32" or (conv == "x3" and self.wx3) or (
            conv in ("dx3", "dx3w16") and self.dx3)

    def clear_range_flag(self):
        self.range_flag.zero_()

    def range_flag_tripped(self) -> bool:
        return bool(self.range_flag.item())

    # ------------------------------------------------------------ geometry
    def sym_offsets(self, B: int) -> list[int]:
        """start of each level's block in the flat latent buffers"""
        offs, o = [], 0
        for L in self.levels:
            offs.append(o)
            o += B * L.n_sym
        offs.append(o)
        return offs

    def flops_per_image(self, fold: bool = False) -> dict:
        """FLOPs of one image per direction (unpadded): fold=False as the reference
        computes the flow; fold=True as this engine does when it folds the 1x1 convs."""
        c = p = 0
        for l, L in enumerate(self.levels):
            hw = L.h * L.w
            c += hw * sum(b.geom.flops_per_pixel(fold) for b in self.couple[l])
            p += hw * self.prior[l].geom.flops_per_pixel(fold)
        return {"couple": c, "prior": p, "total": c + p}

    # ------------------------------------------------------------ workspace
    def workspace(self, B: int, slot: int = 0):
        """Activation / latent buffers for B images.  Each slot is an independent set (the
        ImageCodec lanes run one slot per HIP stream); the ws_keep most recently used sets stay
        resident (ImageCodec raises ws_keep to its lanes + the pipelined encode's slot + 1)."""
        ws = self._ws.get((B, slot))
        if ws is not None:
            self._ws.move_to_end((B, slot))  # least recently used goes first
            return ws
        dev = self.device
        f = lambda n: torch.empty(int(n), dtype=torch.float32, device=dev)  # noqa: E731
        Pmax = max(B * L.h * L.w for L in self.levels)
        ws = {
            "img": f(B * self.H * self.W * 4),
            "x": [[f(B * L.h * L.w * L.ldx), f(B * L.h * L.w * L.ldx)] for L in self.levels],
            "feat": f(Pmax * self.ld_feat),
            "tmp": f(self._tmp_floats(B)),
            "lat": f(B * self.n_sym_img),
            "mean": f(B * self.n_sym_img),
            "logscale": f(B * self.n_sym_img),
            "scale": f(B * self.n_sym_img),
            "cur": [0] * self.nsplit,
        }
        if self.conditional:
            ws["cond"] = [f(B * L.h * L.w * round_up(L.cond_ch, 4)) for L in self.levels]
            # channels C..3 of the 4-wide pixel rows stay zero (they meet zero weights)
            ws["cond_img"] = torch.zeros(B * self.H * self.W * 4, dtype=torch.float32, device=dev)
        # the last few sets stay resident (an encode batch plus the decode lanes' sub-batches)
        while len(self._ws) >= max(1, self.ws_keep):
            self._ws.pop(next(iter(self._ws)))
        self._ws[(B, slot)] = ws
        return ws

    def _tmp_floats(self, B: int) -> int:
        """Floats of a workspace's tmp: P * ld_tmp at the widest level, and at every level room
        for the dx3 layers' split copy (<= P * ld_tmp) plus their split-K workspace
        (idf_conv3x3_dx3_workspace: the 8 x 8 level's partial sums)."""
        n = 0
        for l, Lv in enumerate(self.levels):
            P = B * Lv.h * Lv.w
            extra = 0
            for b in self.couple[l] + [self.prior[l]]:
                nd = len(b.dx3_w) or len(b.dxb_w)  # dxb: every layer (the bf16 shadow's tail)
                if nd:
                    w = lib().idf_conv3x3_dx3_workspace(B, Lv.h, Lv.w, b.geom.k_in[nd - 1],
                                                        b.geom.g_pad)
                    extra = max(extra, int(w))
            # + the fused head's running sums [P][16] (and the split-K workspace)
            n = max(n, P * self.ld_tmp + (extra + 512) // 4 + 32 * P)
            # at least what the library lays out for each block as currently set up (the split
            # copy, split-K workspace and head sums: idf_dense_block_dx3_tmp_bytes)
            for b in self.couple[l] + [self.prior[l]]:
                nb = int(lib().idf_dense_block_dx3_tmp_bytes(ctypes.byref(b.desc), B, Lv.h, Lv.w))
                if nb < 0:
                    raise IdfError(f"dense block tmp size query failed at level {l}")
                n = max(n, (nb + 255) // 4)
        return n

    def tmp_pitch(self, ws, P: int) -> int:
        """ld_tmp for a dense block of P pixels in ws['tmp']: the whole buffer as P rows (a
        multiple of 16 floats), so the block sees every byte of it."""
        return max(self.ld_tmp, (ws["tmp"].numel() // max(P, 1)) // 16 * 16)

    # ------------------------------------------------------------ pieces
    def _x(self, ws, l, which=0):
        return ws["x"][l][(ws["cur"][l] + which) % 2]

    def _swap(self, ws, l):
        ws["cur"][l] ^= 1

    def _prep_cond(self, ws, B, cond_nchw, s):
        """ConditionalFlows cond at each level: ExtendDim of the cond image
        (flows.py:309) or the stride-2 convs (flows.py:310-313)."""
        L = lib()
        check(L.idf_nchw_to_pm(s, B, self.C, self.H, self.W, ptr(cond_nchw), ptr(ws["cond_img"]), 4),
              "nchw_to_pm")
        src, ld, H, W, C = ws["cond_img"], 4, self.H, self.W, self.C
        for l, Lv in enumerate(self.levels):
            dst, ldd = ws["cond"][l], round_up(Lv.cond_ch, 4)
            if self.conv_for_cond:
                dc = self.cond_conv[l]
                c = dc.c
                check(L.idf_conv_taps_f32(s, B, H, W, round_up(C, 4), ptr(src), ld, H // 2, W // 2,
                                          2, 2, len(c.dy), dc.dy, dc.dx, ptr(dc.w), c.ldw,
                                          c.n_alloc, ptr(dc.b), Lv.cond_ch, ptr(dst), ldd, H // 2,
                                          W // 2, 1, 1, 0, 0, None, 0, _lib.ACT["None"], 0.0),
                      "cond conv")
            else:
                check(L.idf_squeeze(s, B, H, W, C, self.scale, ptr(src), ld, ptr(dst), ldd),
                      "squeeze")
            src, ld, H, W, C = dst, ldd, Lv.h, Lv.w, Lv.cond_ch

    def _prior(self, ws, B, l, s, mean, logscale, scale, x_src=None, ld_src=0):
        """Prior.forward (priorlib.py:36-47) on pixel-major input written into feat."""
        L = lib()
        Lv = self.levels[l]
        blk = self.prior[l]
        P = B * Lv.h * Lv.w
        feat = ws["feat"]
        ld = self.ld_feat
        nx = Lv.C if Lv.prior_x_zero else Lv.rest
        a_pad = blk.geom.a_pad
        if self.conditional:
            if Lv.prior_x_zero:
                check(L.idf_copy_cols(s, P, 0, nx, None, 0, ptr(feat), ld), "zero cols")
            else:
                check(L.idf_copy_cols(s, P, nx, nx, x_src, ld_src, ptr(feat), ld), "copy cols")
            check(L.idf_copy_cols(s, P, Lv.cond_ch, a_pad - nx, ptr(ws["cond"][l]),
                                  round_up(Lv.cond_ch, 4), ptr(feat) + nx * FLOAT, ld), "cond cols")
        elif Lv.prior_x_zero:
            check(L.idf_copy_cols(s, P, 0, a_pad, None, 0, ptr(feat), ld), "zero cols")
        else:
            check(L.idf_copy_cols(s, P, nx, a_pad, x_src, ld_src, ptr(feat), ld), "copy cols")
        blk.run(s, B, Lv.h, Lv.w, ptr(feat), ld, ptr(ws["tmp"]), self.tmp_pitch(ws, P),
                head_prior(Lv.z, mean, logscale, scale))

    def ensure_top_prior(self, ws, s):
        """Computes the cached top prior on stream s if it is needed and missing (the lanes
        call this on their parent stream before forking, so no lane races its creation)."""
        Lv = self.levels[-1]
        if self.conv_mode not in self._top_prior and Lv.prior_x_zero and not self.conditional:
            self._top_prior_cached(ws, 0, s, 0)

    def _top_prior_cached(self, ws, B, s, off):
        """IDFlows' top prior sees zeros (priorlib.py:43): its output does not depend on
        the data, so it is computed once per conv mode (batch 1) and replicated per image;
        the entry lives as long as the engine (see __init__)."""
        Lv = self.levels[-1]
        n = Lv.n_sym
        hit = self._top_prior.get(self.conv_mode)
        if hit is None:
            t = torch.empty(3 * n, dtype=torch.float32, device=self.device)
            ws1 = {"feat": ws["feat"], "tmp": ws["tmp"]}
            self._prior(ws1, 1, self.nsplit - 1, s, ptr(t), ptr(t) + n * FLOAT,
                        ptr(t) + 2 * n * FLOAT)
            made = torch.cuda.Event()
            made.record()  # the stream it was computed on (current: s)
            hit = self._top_prior[self.conv_mode] = (t.view(3, n), made)
        tp, made = hit
        # a user on another stream (the other side of a pipelined encode / decode) waits for
        # the computation, wherever it was enqueued
        torch.cuda.current_stream(self.device).wait_event(made)
        for i, key in enumerate(("mean", "logscale", "scale")):
            ws[key][off: off + B * n].view(B, n).copy_(tp[i].expand(B, n))

    # ------------------------------------------------------------ forward
    @torch.no_grad()
    def forward_pm(self, B: int, cond=None, slot: int = 0, on_level=None):
        """Runs flows.py:87-116 from ws['img'] (pixel-major, ld 4) for B images.
        Fills ws lat/mean/logscale/scale.  Returns the workspace."""
        gen = self.forward_pm_steps(B, cond=cond, slot=slot, on_level=on_level)
        while True:
            try:
                next(gen)
            except StopIteration as done:
                return done.value

    def forward_pm_steps(self, B: int, cond=None, slot: int = 0, on_level=None):
        """forward_pm as a generator that yields after each coupling block and after each
        level's prior (and on_level), so that the host can interleave the enqueue of several
        encode lanes (ImageCodec): all launches go to the stream current at the FIRST step.
        Returns (StopIteration.value) the workspace."""
        L = lib()
        ws = self.workspace(B, slot)
        s = _lib.stream_ptr(self.device)
        offs = self.sym_offsets(B)
        if self.conditional:
            self._prep_cond(ws, B, cond, s)
        src, ld_src, H, W, C = ptr(ws["img"]), 4, self.H, self.W, self.C
        for l, Lv in enumerate(self.levels):
            ws["cur"][l] = 0
            P = B * Lv.h * Lv.w
            check(L.idf_squeeze(s, B, H, W, C, self.scale, src, ld_src, ptr(self._x(ws, l)), Lv.ldx),
                  "squeeze")
            for k in range(self.nflows):
                blk = self.couple[l][k]
                x, x2 = self._x(ws, l), self._x(ws, l, 1)
                check(L.idf_permute_couple_in(s, P, Lv.C, ptr(self.ids[l][k]), ptr(x), Lv.ldx, ptr(x2),
                                              Lv.ldx, Lv.a, blk.geom.a_pad, ptr(ws["feat"]),
                                              self.ld_feat), "permute")
                self._swap(ws, l)
                xo = ptr(x2) + Lv.a * FLOAT
                blk.run(s, B, Lv.h, Lv.w, ptr(ws["feat"]), self.ld_feat, ptr(ws["tmp"]),
                        self.tmp_pitch(ws, P), head_couple(_lib.EPI_COUPLE_ADD, xo, Lv.ldx))
                yield l
            x, x2 = self._x(ws, l), self._x(ws, l, 1)
            check(L.idf_permute_couple_in(s, P, Lv.C, ptr(self.ids[l][self.nflows]), ptr(x), Lv.ldx,
                                          ptr(x2), Lv.ldx, 0, 0, None, 0), "permute")
            self._swap(ws, l)
            x = self._x(ws, l)
            o = offs[l]
            check(L.idf_pm_to_nchw(s, B, Lv.z, Lv.h, Lv.w, ptr(x), Lv.ldx,
                                   ptr(ws["lat"]) + o * FLOAT), "pm_to_nchw")
            mean, logs, scale = (ptr(ws[k]) + o * FLOAT for k in ("mean", "logscale", "scale"))
            if Lv.prior_x_zero and not self.conditional:
                self._top_prior_cached(ws, B, s, o)
            else:
                self._prior(ws, B, l, s, mean, logs, scale, ptr(x) + Lv.z * FLOAT, Lv.ldx)
            if on_level is not None:  # level l's lat / mean / scale are final
                on_level(l, ws)
            yield l
            src, ld_src, H, W, C = ptr(x) + Lv.z * FLOAT, Lv.ldx, Lv.h, Lv.w, Lv.rest
        return ws

    def load_u8(self, img_u8: torch.Tensor, slot: int = 0):
        B = img_u8.shape[0]
        ws = self.workspace(B, slot)
        check(lib().idf_dequant_u8(_lib.stream_ptr(self.device), B, self.C, self.H, self.W,
                                   ptr(img_u8), ptr(ws["img"]), 4), "dequant")
        return ws

    def load_nchw(self, x: torch.Tensor, slot: int = 0):
        B = x.shape[0]
        ws = self.workspace(B, slot)
        x = x.contiguous().float()
        check(lib().idf_nchw_to_pm(_lib.stream_ptr(self.device), B, self.C, self.H, self.W, ptr(x),
                                   ptr(ws["img"]), 4), "nchw_to_pm")
        return ws

    # ------------------------------------------------------------ inverse
    @torch.no_grad()
    def inverse_pm(self, B: int, decode_level, cond=None, priors: bool = True, slot: int = 0):
        """Top-down decoder (flows.py:118-152 order).  For each level l (top first):
        prior -> decode_level(l, ws) fills ws['lat'] level l -> flows backward ->
        unsqueeze.  The image lands in ws['img'] (pixel-major, ld 4)."""
        steps = self.inverse_pm_steps(B, decode_level, cond, priors, slot)
        while True:
            try:
                next(steps)
            except StopIteration as done:
                return done.value

    def inverse_pm_steps(self, B: int, decode_level, cond=None, priors: bool = True,
                         slot: int = 0, pre_prior=None):
        """inverse_pm as a generator that yields after each level's decode_level and after
        each coupling block, so that the host can interleave the enqueue of several decode
        lanes (ImageCodec): all launches go to the stream current at the FIRST step.  Its
        return value (StopIteration.value) is the workspace it decoded into -- the caller must
        use that one, not look the slot up again (the cache may have evicted the key).
        pre_prior(l), if given, is called just before level l's prior is enqueued."""
        L = lib()
        ws = self.workspace(B, slot)
        s = _lib.stream_ptr(self.device)
        offs = self.sym_offsets(B)
        if self.conditional and priors:
            self._prep_cond(ws, B, cond, s)
        for l in reversed(range(self.nsplit)):
            Lv = self.levels[l]
            P = B * Lv.h * Lv.w
            x = self._x(ws, l)
            o = offs[l]
            if pre_prior is not None:
                pre_prior(l)
            if priors:
                mean, logs, scale = (ptr(ws[k]) + o * FLOAT for k in ("mean", "logscale", "scale"))
                if Lv.prior_x_zero and not self.conditional:
                    self._top_prior_cached(ws, B, s, o)
                else:
                    self._prior(ws, B, l, s, mean, logs, scale, ptr(x) + Lv.z * FLOAT, Lv.ldx)
            decode_level(l, ws)
            yield l
            check(L.idf_nchw_to_pm(s, B, Lv.z, Lv.h, Lv.w, ptr(ws["lat"]) + o * FLOAT, ptr(x),
                                   Lv.ldx), "nchw_to_pm")
            x2 = self._x(ws, l, 1)
            check(L.idf_permute_couple_in(s, P, Lv.C, ptr(self.inv_ids[l][self.nflows]), ptr(x),
                                          Lv.ldx, ptr(x2), Lv.ldx, 0, 0, None, 0), "permute")
            self._swap(ws, l)
            for k in reversed(range(self.nflows)):
                blk = self.couple[l][k]
                x, x2 = self._x(ws, l), self._x(ws, l, 1)
                check(L.idf_copy_cols(s, P, Lv.a, blk.geom.a_pad, ptr(x), Lv.ldx, ptr(ws["feat"]),
                                      self.ld_feat), "copy cols")
                xo = ptr(x) + Lv.a * FLOAT
                blk.run(s, B, Lv.h, Lv.w, ptr(ws["feat"]), self.ld_feat, ptr(ws["tmp"]),
                        self.tmp_pitch(ws, P), head_couple(_lib.EPI_COUPLE_SUB, xo, Lv.ldx))
                check(L.idf_permute_couple_in(s, P, Lv.C, ptr(self.inv_ids[l][k]), ptr(x), Lv.ldx,
                                              ptr(x2), Lv.ldx, 0, 0, None, 0), "permute")
                self._swap(ws, l)
                yield l
            x = self._x(ws, l)
            if l > 0:
                Lp = self.levels[l - 1]
                dst, ldd = ptr(self._x(ws, l - 1)) + Lp.z * FLOAT, Lp.ldx
                Hh, Ww, Cc = Lp.h, Lp.w, Lp.rest
            else:
                dst, ldd, Hh, Ww, Cc = ptr(ws["img"]), 4, self.H, self.W, self.C
            check(L.idf_unsqueeze(s, B, Hh, Ww, Cc, self.scale, ptr(x), Lv.ldx, dst, ldd),
                  "unsqueeze")
        return ws

    def image_nchw(self, ws, B, out=None):
        if out is None:
            out = torch.empty((B, self.C, self.H, self.W), dtype=torch.float32, device=self.device)
        check(lib().idf_pm_to_nchw(_lib.stream_ptr(self.device), B, self.C, self.H, self.W,
                                   ptr(ws["img"]), 4, ptr(out)), "pm_to_nchw")
        return out

    def image_u8(self, ws, B, out=None, bad=None):
        """ws['img'] -> uint8 NCHW (out: a contiguous [B, C, H, W] view to fill) and the
        off-grid pixel count (added into bad)."""
        if out is None:
            out = torch.empty((B, self.C, self.H, self.W), dtype=torch.uint8, device=self.device)
        if bad is None:
            bad = torch.zeros(1, dtype=torch.int32, device=self.device)
        check(lib().idf_quant_u8(_lib.stream_ptr(self.device), B, self.C, self.H, self.W,
                                 ptr(ws["img"]), 4, ptr(out), ptr(bad)), "quant")
        return out, bad

    def level_views(self, ws, B, key):
        offs = self.sym_offsets(B)
        return [ws[key][offs[l]: offs[l + 1]].view(B, L.z, L.h, L.w)
                for l, L in enumerate(self.levels)]

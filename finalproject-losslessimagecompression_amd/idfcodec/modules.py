"""Module-level device forward of the reference building blocks (NCHW in, NCHW out).

The model-level path (FlowEngine) keeps activations pixel-major end to end;
these helpers serve the reference's per-module API (DenseLayer.forward,
DenseBlock.forward, AdditiveCouple.forward/backward, Prior.forward) and the
teacher-forced parity tests.  Every call goes through libidfcodec.so.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import IdfHeadOut, check, lib, ptr, require_device
from .engine import FLOAT, DeviceBlock, head_couple, head_prior
from .packing import pack_dense_block, round_up


def _param_key(module):
    return tuple((p.data_ptr(), p._version) for p in module.parameters())


def device_block(block, device, fold=None) -> DeviceBlock:
    """Packed DeviceBlock of a DenseBlock module, cached until its parameters change.
    fold: fold the 1x1 convs into the 3x3 convs (default: engine.FOLD)."""
    from .engine import FOLD
    fold = FOLD if fold is None else bool(fold)
    key = (_param_key(block), str(device), fold)
    cached = getattr(block, "_idf_device_block", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    sd = {k: v for k, v in block.state_dict().items()}
    db = DeviceBlock(pack_dense_block(sd, "", block.depth, block.act_name, fold=fold), device)
    object.__setattr__(block, "_idf_device_block", (key, db))
    return db


def _layer_as_block(layer, device) -> DeviceBlock:
    key = (_param_key(layer), str(device))
    cached = getattr(layer, "_idf_device_block", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    c, o = layer.i_channel, layer.o_channel
    sd = {
        "layers.0.layers.0.weight": layer.layers[0].weight, "layers.0.layers.0.bias": layer.layers[0].bias,
        "layers.0.layers.1.weight": layer.layers[1].weight, "layers.0.layers.1.bias": layer.layers[1].bias,
        "layers.1.weight": torch.zeros(1, o, 1, 1), "layers.1.bias": torch.zeros(1),
    }
    db = DeviceBlock(pack_dense_block(sd, "", 1, layer.act_name), device)
    object.__setattr__(layer, "_idf_device_block", (key, db))
    return db


def _feat_from_nchw(x, db: DeviceBlock, extra_cols=0):
    B, C, H, W = x.shape
    P = B * H * W
    ld = db.geom.ld_feat
    feat = torch.zeros(P * ld, dtype=torch.float32, device=x.device)
    s = _lib.stream_ptr(x.device)
    check(lib().idf_nchw_to_pm(s, B, C, H, W, ptr(x.contiguous().float()), ptr(feat), ld), "nchw_to_pm")
    return feat, ld, s


def dense_tmp(db: DeviceBlock, B: int, H: int, W: int, ld_tmp: int, device):
    """(tmp, its pitch) for one dense block run: P x ld_tmp floats, plus the dx3 / dxb layers'
    split-K workspace where the geometry splits (idf_conv3x3_dx3_workspace)."""
    P = B * H * W
    n = P * ld_tmp
    # dx3 / dxb: + the split-K workspace and the fused head's sums [P][16]
    nd = len(db.dx3_w) if db.desc.dx3 else (len(db.dxb_w) if db.desc.dxb else 0)
    if nd:
        w = int(lib().idf_conv3x3_dx3_workspace(B, H, W, db.geom.k_in[nd - 1], db.geom.g_pad))
        n += (max(w, 0) + 512) // 4 + 32 * P
    tmp = torch.empty(n, dtype=torch.float32, device=device)
    return tmp, max(ld_tmp, (n // P) // 16 * 16)


@torch.no_grad()
def run_dense_block(block, x: torch.Tensor, fold=None) -> torch.Tensor:
    """DenseBlock.forward (nnblock.py:53-56) -> NCHW [B, o_channel, H, W]."""
    require_device(x, "DenseBlock input")
    return run_device_block(device_block(block, x.device, fold), x)[0]


@torch.no_grad()
def run_device_block(db: DeviceBlock, x: torch.Tensor, return_feat: bool = False):
    """A packed DeviceBlock -- e.g. one of a FlowEngine's own coupling / prior blocks, in
    the engine's conv mode -- over NCHW input x: (head output NCHW [B, n_head, H, W], the
    pixel-major feature buffer [P, ld_feat] holding the input and every layer's output, or
    None unless return_feat)."""
    require_device(x, "DenseBlock input")
    B, C, H, W = x.shape
    feat, ld, s = _feat_from_nchw(x, db)
    P = B * H * W
    ld_tmp = ld
    if db.desc.bf16:  # bf16 shadow of the features ahead of the split-K partials
        ld_tmp = max(ld, round_up(ld, 64) // 2 + 2 * 48 + 8)
    tmp, ld_tmp = dense_tmp(db, B, H, W, ld_tmp, x.device)
    n = db.geom.n_head
    ldo = round_up(n, 4)
    out_pm = torch.empty(B * H * W * ldo, dtype=torch.float32, device=x.device)
    # the head inside the block call with a plain store epilogue -- fused into the dx3 layers
    # where the engine fuses it, else the head GEMM -- and, for return_feat, the layers' fp32
    # outputs kept (a fused head otherwise drops them)
    head = IdfHeadOut()
    head.mode = _lib.EPI_STORE
    head.out = ptr(out_pm)
    head.ld_out = ldo
    keep = db.desc.keep_feat
    db.desc.keep_feat = 1 if return_feat else keep
    try:
        check(lib().idf_dense_block_f32(s, ctypes.byref(db.desc), B, H, W, ptr(feat), ld,
                                        ptr(tmp), ld_tmp, ctypes.byref(head)), "dense block")
    finally:
        db.desc.keep_feat = keep
    out = torch.empty((B, n, H, W), dtype=torch.float32, device=x.device)
    check(lib().idf_pm_to_nchw(s, B, n, H, W, ptr(out_pm), ldo, ptr(out)), "pm_to_nchw")
    return out, (feat.view(P, ld) if return_feat else None)


@torch.no_grad()
def run_dense_layer(layer, x: torch.Tensor) -> torch.Tensor:
    """DenseLayer.forward (nnlayer.py:48-51) -> NCHW cat(x, act(conv3(conv1(x))))."""
    require_device(x, "DenseLayer input")
    db = _layer_as_block(layer, x.device)
    B, C, H, W = x.shape
    feat, ld, s = _feat_from_nchw(x, db)
    tmp = torch.empty_like(feat)
    g = db.geom
    check(lib().idf_conv1x1_f32(s, B * H * W, g.k_in[0], g.k_in[0], ptr(feat), ld, ptr(db.w1[0]),
                                db.packed.ldw1[0], db.packed.n1_alloc[0], ptr(db.b1[0]), ptr(tmp), ld,
                                B, H, W, None), "conv1x1")
    check(lib().idf_conv3x3_f32(s, B, H, W, g.k_in[0], ptr(tmp), ld, ptr(db.w3[0]),
                                db.packed.ldw3[0], db.packed.g_alloc, ptr(db.b3[0]), g.g_pad,
                                ptr(feat) + g.k_in[0] * FLOAT, ld, _lib.ACT[db.packed.act],
                                db.packed.slope), "conv3x3")
    pos = torch.as_tensor(g.positions(layer.o_channel), device=x.device)
    fm = feat.view(B * H * W, ld)[:, pos]
    return fm.view(B, H, W, layer.o_channel).permute(0, 3, 1, 2).contiguous()


@torch.no_grad()
def run_couple(couple, x: torch.Tensor, sign: int) -> torch.Tensor:
    """AdditiveCouple.forward (sign=+1, couplelib.py:47-53) / backward (sign=-1, :55-61)."""
    require_device(x, "AdditiveCouple input")
    db = device_block(couple.dense, x.device)
    B, C, H, W = x.shape
    P = B * H * W
    ldx = round_up(C, 4)
    s = _lib.stream_ptr(x.device)
    xpm = torch.empty(P * ldx, dtype=torch.float32, device=x.device)
    check(lib().idf_nchw_to_pm(s, B, C, H, W, ptr(x.contiguous().float()), ptr(xpm), ldx), "nchw_to_pm")
    ld = db.geom.ld_feat
    feat = torch.empty(P * ld, dtype=torch.float32, device=x.device)
    tmp, ld_tmp = dense_tmp(db, B, H, W, ld, x.device)
    check(lib().idf_copy_cols(s, P, couple.a_ch, db.geom.a_pad, ptr(xpm), ldx, ptr(feat), ld), "copy")
    mode = _lib.EPI_COUPLE_ADD if sign > 0 else _lib.EPI_COUPLE_SUB
    db.run(s, B, H, W, ptr(feat), ld, ptr(tmp), ld_tmp,
           head_couple(mode, ptr(xpm) + couple.a_ch * FLOAT, ldx))
    out = torch.empty((B, C, H, W), dtype=torch.float32, device=x.device)
    check(lib().idf_pm_to_nchw(s, B, C, H, W, ptr(xpm), ldx, ptr(out)), "pm_to_nchw")
    return out


@torch.no_grad()
def run_prior(prior, inp: torch.Tensor):
    """Prior.forward (priorlib.py:36-47) -> (mean, logscale) NCHW."""
    require_device(inp, "Prior input")
    db = device_block(prior.NN, inp.device)
    x = inp if prior.cond_channel > 0 else torch.zeros_like(inp)
    B, C, H, W = x.shape
    feat, ld, s = _feat_from_nchw(x, db)
    tmp, ld_tmp = dense_tmp(db, B, H, W, ld, x.device)
    n = prior.out_channel
    mean = torch.empty((B, n, H, W), dtype=torch.float32, device=x.device)
    logs = torch.empty_like(mean)
    scale = torch.empty_like(mean)
    db.run(s, B, H, W, ptr(feat), ld, ptr(tmp), ld_tmp,
           head_prior(n, ptr(mean), ptr(logs), ptr(scale)))
    return mean, logs

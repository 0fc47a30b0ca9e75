"""Lossless codec of the residual configs (configs 3-5; trainer.py:550-801 ResidualTrainer).

encode (trainer.py:603-621, made lossless):
  u8 -> data on the 1/256 grid (trainer.py:101) -> VQ-VAE indices (vqvae.py:135-147) ->
  rec = round8(decoder(embed[idx]) * 0.5 + 0.5) (trainer.py:606-607) -> res = data - rec
  (:608) -> Patching (extenddim.py:52-58) of res and rec -> the flow model's forward with
  cond = rec patches (ConditionalFlows) -> rANS streams.
  The VQ indices travel too, as a fixed-width code of ceil(log2(embed_num)) bits each --
  the reference counts only the residual's bits (trainer.py:698-701) and never codes the
  indices; bits() reports both parts.
decode: indices -> rec (the same device function as the encoder side) -> flow decode with
  cond = rec patches -> unpatch -> data = res + rec -> uint8 (exact on the grid).
"""
from __future__ import annotations

import math
import struct
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr
from .codec import Bitstream, ImageCodec

MAGIC = b"IDFR"
VERSION = 2         # 2 adds the source (pre-pad) image size; version-1 streams still read
# header flags bit 0: the VQ decoder's 3x3 convs ran as split-f16 products (vq_conv "x3");
# 0: exact-f32 Winograd (every stream written before the field existed)
FLAG_VQ_X3 = 1
# bit 1 (with bit 0): the other VQ convs ran as split-f16 products too (vq_conv "x3t",
# idf_conv_taps_x3); absent in files written before round 6
FLAG_VQ_TAPS = 2


@dataclass
class ResidualBitstream:
    flow: Bitstream
    idx_words: torch.Tensor     # int32 view of the packed index words (image-aligned runs)
    n_images: int
    image_shape: tuple          # (C, H, W)
    grid: tuple                 # (h, w) of the VQ indices per image
    embed_num: int
    source_hw: tuple | None = None   # (H, W) before the dataloader's replication pad
    vq_conv: str = "f32"        # the VQ decoder's conv arithmetic (idfcodec.vq.VQEngine)

    @property
    def source_shape(self) -> tuple:
        C, H, W = self.image_shape
        return (C,) + tuple(self.source_hw or (H, W))

    @property
    def index_bits(self) -> int:
        return max(1, math.ceil(math.log2(self.embed_num)))

    def bits(self) -> int:
        """flow streams (the reference's accounting, trainer.py:326-327) + index code"""
        return self.flow.bits() + self.n_images * self.grid[0] * self.grid[1] * self.index_bits

    def bpd(self) -> float:
        C, H, W = self.image_shape
        return self.bits() / (self.n_images * C * H * W)

    def to_bytes(self) -> bytes:
        C, H, W = self.image_shape
        sh, sw = self.source_hw or (H, W)
        if self.vq_conv not in ("x3t", "x3", "f32"):
            raise ValueError(f"unknown VQ conv mode {self.vq_conv!r}")
        flags = {"x3t": FLAG_VQ_X3 | FLAG_VQ_TAPS, "x3": FLAG_VQ_X3, "f32": 0}[self.vq_conv]
        hdr = struct.pack("<4sHHIIIIIIIII", MAGIC, VERSION, flags, self.n_images, C, H, W,
                          self.grid[0], self.grid[1], self.embed_num, sh, sw)
        iw = self.idx_words.detach().cpu().numpy().astype("<i4").tobytes()
        fb = self.flow.to_bytes()
        return hdr + struct.pack("<QQ", len(iw), len(fb)) + iw + fb

    @classmethod
    def from_bytes(cls, buf: bytes, device=None) -> "ResidualBitstream":
        fmt = "<4sHHIIIIIII"
        magic, ver, _f, n, C, H, W, h, w, K = struct.unpack_from(fmt, buf, 0)
        if magic != MAGIC or ver not in (1, VERSION):
            raise ValueError("not an IDF residual bitstream")
        if _f & ~(FLAG_VQ_X3 | FLAG_VQ_TAPS) or (_f & FLAG_VQ_TAPS and not _f & FLAG_VQ_X3):
            raise ValueError(f"unknown residual bitstream flags {_f:#x}")
        o = struct.calcsize(fmt)
        src = None
        if ver >= 2:
            src = struct.unpack_from("<II", buf, o)
            o += 8
        li, lf = struct.unpack_from("<QQ", buf, o)
        o += 16
        iw = np.frombuffer(buf, "<i4", li // 4, o).copy()
        o += li
        flow = Bitstream.from_bytes(buf[o:o + lf], device)
        t = torch.from_numpy(iw)
        return cls(flow, t.to(device) if device else t, n, (C, H, W), (h, w), K,
                   None if src is None or tuple(src) == (H, W) else tuple(src),
                   "x3t" if _f & FLAG_VQ_TAPS else ("x3" if _f & FLAG_VQ_X3 else "f32"))


class ResidualCodec:
    """uint8 images <-> ResidualBitstream with a flow model (ConditionalFlows or IDFlows)
    over Patching(input_size -> model H x W) and a VQ-VAE.

    pad = (bottom, right): the dataloader's ReplicationPad2d (trainer.py:62), applied on the
    device to images of size input_size - pad before coding and cropped off after decoding,
    so the source image comes back exactly.  Images already of input_size are coded as is."""

    def __init__(self, flows_model, vqvae, input_size, pad=(0, 0)):
        from extenddim import Patching
        self.flows = flows_model
        self.vqvae = vqvae
        self.H, self.W = int(input_size[0]), int(input_size[1])
        self.patch = Patching(self.H, self.W, flows_model.H, flows_model.W)
        self.conditional = type(flows_model).__name__ == "ConditionalFlows"
        self.bits = max(1, math.ceil(math.log2(vqvae.embed_num)))
        self.pad = (int(pad[0]), int(pad[1]))
        # bench timing (tools/bench_residual.py): when a list, encode / decode append
        # (phase name, HIP event) at each phase's end on the current stream
        self.phases = None

    def _mark(self, name):
        if self.phases is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.phases.append((name, e))

    @staticmethod
    def _edge(img_u8, Ho, Wo):
        B, C, H, W = img_u8.shape
        if (H, W) == (Ho, Wo):
            return img_u8
        out = torch.empty((B, C, Ho, Wo), dtype=torch.uint8, device=img_u8.device)
        check(lib().idf_pad_edge_u8(_lib.stream_ptr(img_u8.device), B, C, H, W, Ho, Wo,
                                    ptr(img_u8), ptr(out)), "pad/crop")
        return out

    def _codec(self) -> ImageCodec:
        return self.flows.codec()

    def _dequant(self, img_u8):
        B, C, H, W = img_u8.shape
        dev = img_u8.device
        s = _lib.stream_ptr(dev)
        pm = torch.empty(B * H * W * 4, dtype=torch.float32, device=dev)
        check(lib().idf_dequant_u8(s, B, C, H, W, ptr(img_u8), ptr(pm), 4), "dequant")
        out = torch.empty((B, C, H, W), dtype=torch.float32, device=dev)
        check(lib().idf_pm_to_nchw(s, B, C, H, W, ptr(pm), 4, ptr(out)), "pm->nchw")
        return out

    @staticmethod
    def _pointwise(op, x, z):
        out = torch.empty_like(x)
        n = x.numel()
        check(lib().idf_vq_pointwise(_lib.stream_ptr(x.device), n, 1, op, ptr(x), 1, ptr(z), 1,
                                     ptr(out), 1), "pointwise")
        return out

    @torch.no_grad()
    def encode(self, img_u8: torch.Tensor) -> ResidualBitstream:
        _lib.require_device(img_u8, "image batch")
        if img_u8.dtype != torch.uint8:
            raise TypeError("ResidualCodec.encode expects uint8 images")
        img_u8 = img_u8.contiguous()
        src_hw = tuple(img_u8.shape[2:])
        if src_hw == (self.H - self.pad[0], self.W - self.pad[1]):
            img_u8 = self._edge(img_u8, self.H, self.W)
        B, C, H, W = img_u8.shape
        if (H, W) != (self.H, self.W):
            raise ValueError(f"image size {src_hw}: the codec takes {(self.H, self.W)}"
                             + (f" or {(self.H - self.pad[0], self.W - self.pad[1])}"
                                if any(self.pad) else ""))
        self._mark("start")
        data = self._dequant(img_u8)
        self._mark("pad_dequant")
        idx = self.vqvae.indices(data)                       # [B, h, w] int32
        self._mark("vq_indices")
        rec = self.vqvae.reconstruct(idx)                    # NCHW on the grid
        self._mark("vq_reconstruct")
        vq_conv = self.vqvae.engine().last_decode_mode       # what the receiver must run
        res = self._pointwise(2, data, rec)                  # data - rec
        res_p, _ = self.patch.forward(res, None)
        codec = self._codec()
        if self.conditional:
            rec_p, _ = self.patch.forward(rec, None)
            self._mark("residual_patching")
            flow = codec.encode_nchw(res_p, cond=rec_p.contiguous())
        else:
            self._mark("residual_patching")
            flow = codec.encode_nchw(res_p)
        self._mark("flow_encode")
        per = idx.shape[1] * idx.shape[2]
        nwd = int(lib().idf_pack_bits_words(B, per, self.bits))
        words = torch.empty(max(nwd, 1), dtype=torch.int32, device=img_u8.device)
        check(lib().idf_pack_bits(_lib.stream_ptr(img_u8.device), B, per, self.bits, ptr(idx),
                                  ptr(words)), "pack idx")
        words = words[:nwd]
        self._mark("index_code")
        return ResidualBitstream(flow, words, B, (C, H, W), tuple(idx.shape[1:]),
                                 self.vqvae.embed_num, None if src_hw == (H, W) else src_hw,
                                 vq_conv)

    @torch.no_grad()
    def decode(self, rbs: ResidualBitstream, verify: bool = True):
        dev = next(self.flows.parameters()).device
        B = rbs.n_images
        C, H, W = rbs.image_shape
        h, w = rbs.grid
        n = B * h * w
        words = rbs.idx_words.to(dev)
        if words.numel() == 0:
            words = torch.zeros(1, dtype=torch.int32, device=dev)
        idx = torch.empty(n, dtype=torch.int32, device=dev)
        self._mark("start")
        check(lib().idf_unpack_bits(_lib.stream_ptr(dev), B, h * w, self.bits, ptr(words),
                                    ptr(idx)), "unpack idx")
        self._mark("index_code")
        rec = self.vqvae.reconstruct(idx.view(B, h, w), conv=rbs.vq_conv)
        self._mark("vq_reconstruct")
        codec = self._codec()
        if self.conditional:
            rec_p, _ = self.patch.forward(rec, None)
            self._mark("patching")
            res_p, info = codec.decode_nchw(rbs.flow, cond=rec_p.contiguous(), verify=verify)
        else:
            self._mark("patching")
            res_p, info = codec.decode_nchw(rbs.flow, verify=verify)
        self._mark("flow_decode")
        res = self.patch.backward(res_p.contiguous())
        data = self._pointwise(3, res, rec)                  # res + rec
        s = _lib.stream_ptr(dev)
        pm = torch.empty(B * H * W * 4, dtype=torch.float32, device=dev)
        check(lib().idf_nchw_to_pm(s, B, C, H, W, ptr(data), ptr(pm), 4), "nchw->pm")
        img = torch.empty((B, C, H, W), dtype=torch.uint8, device=dev)
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        check(lib().idf_quant_u8(s, B, C, H, W, ptr(pm), 4, ptr(img), ptr(bad)), "quant")
        if rbs.source_hw:
            img = self._edge(img, *rbs.source_hw)
        self._mark("unpatch_quant_crop")
        info["off_grid"] = bad
        if verify:
            info["ok"] = bool(info.get("ok", True)) and int(bad.item()) == 0
        return img, info

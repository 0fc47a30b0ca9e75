"""ctypes binding of libidfcodec.so (the C ABI declared in include/idf_codec.h).

torch is imported first so that the HIP runtime torch ships (soname
libamdhip64.so.7) is the one libidfcodec.so binds to: device pointers and
stream handles from torch are then valid in the library.

There is no fallback: if the library is missing or no GPU is visible, compute
entry points raise.  Tests on CPU only load the library and inspect exports.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module doc)

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
REPO = os.path.dirname(PKG)
# IDF_LIB_PATH: another build of the same library (same-box A/B runs in tools/ only)
LIB_PATH = os.environ.get("IDF_LIB_PATH") or os.path.join(HERE, "libidfcodec.so")
HEADER = os.path.join(REPO, "include", "idf_codec.h")

IDF_OK = 0
ERR_NAMES = {1: "IDF_ERR_ARG", 2: "IDF_ERR_HIP", 3: "IDF_ERR_WORKSPACE", 4: "IDF_ERR_UNSUPPORTED"}

STREAM_SCALE_ZERO = 1
STREAM_FREQ_ZERO = 2
STREAM_NEG_CDF = 4
STREAM_UNDERFLOW = 8
STREAM_OUT_OF_WINDOW = 16
STREAM_WORDS_LEFT = 32

ACT = {"ReLU": 0, "LeakyReLU": 1, "Tanh": 2, "None": 3}
TAG_CONV1X1, TAG_CONV3X3, TAG_HEAD = 0, 1, 2
EPI_STORE, EPI_COUPLE_ADD, EPI_COUPLE_SUB, EPI_PRIOR = 0, 1, 2, 3
MAX_DEPTH = 32

P = ctypes.c_void_p
i32 = ctypes.c_int32
i64 = ctypes.c_int64
f32 = ctypes.c_float
u64 = ctypes.c_uint64


class IdfDenseBlock(ctypes.Structure):
    _fields_ = [
        ("depth", i32), ("act", i32), ("slope", f32), ("g_pad", i32), ("g_alloc", i32),
        ("k_in", i32 * (MAX_DEPTH + 1)), ("n1_alloc", i32 * MAX_DEPTH), ("ldw1", i32 * MAX_DEPTH),
        ("ldw3", i32 * MAX_DEPTH), ("w1", P * MAX_DEPTH), ("b1", P * MAX_DEPTH),
        ("w3", P * MAX_DEPTH), ("b3", P * MAX_DEPTH), ("n_head", i32), ("nh_alloc", i32),
        ("ldwh", i32), ("wh", P), ("bh", P),
        ("c_real", i32 * (MAX_DEPTH + 1)), ("g_real", i32 * MAX_DEPTH),
        ("fold", i32), ("ldv", i32), ("vtap", P * MAX_DEPTH), ("bfull", P * MAX_DEPTH),
        ("halo", i32), ("wino", i32), ("wino_nft", i32), ("wino_u", P * MAX_DEPTH),
        ("bf16", i32), ("wb16", P * MAX_DEPTH),
        ("wx3", i32), ("wx3_yscale", f32 * MAX_DEPTH), ("wx3_u", P * MAX_DEPTH), ("range_flag", P),
        ("dx3", i32), ("dx3_yscale", f32 * MAX_DEPTH), ("dx3_w", P * MAX_DEPTH),
        ("fuse_head", i32), ("keep_feat", i32),
        ("dxb", i32), ("dxb_w", P * MAX_DEPTH), ("fuse_layers", i32),
    ]


class IdfHeadOut(ctypes.Structure):
    _fields_ = [
        ("mode", i32), ("out", P), ("ld_out", i64), ("base", P), ("ld_base", i64),
        ("n_mean", i32), ("mean", P), ("logscale", P), ("scale", P),
    ]


class IdfDx3Head(ctypes.Structure):
    _fields_ = [
        ("w", P), ("ldw", i32), ("n_head", i32), ("acc", P), ("last", i32), ("skip_f32", i32),
        ("out", IdfHeadOut),
    ]


# name -> (restype, argtypes); mirrors include/idf_codec.h exactly
SIGNATURES = {
    "idf_version": (ctypes.c_char_p, []),
    "idf_device_count": (ctypes.c_int, []),
    "idf_rans_cdf_freq": (ctypes.c_int, [P, i64, P, P, P, P, P]),
    "idf_rans_encode_workspace_bytes": (i64, [i64]),
    "idf_rans_encode_streams": (ctypes.c_int, [P, i64, i64, P, P, P, P, P, P, P, P, P, P, i64]),
    "idf_rans_decode_workspace_bytes": (i64, [i64]),
    "idf_rans_decode_streams": (ctypes.c_int, [P, i64, i64, P, P, P, P, P, P, P, P, P, P, P, i64]),
    "idf_gather_words": (ctypes.c_int, [P, i64, P, P, P, P, P]),
    "idf_rans_host_workspace_bytes": (i64, [i64, i64]),
    "idf_rans_encode_on": (ctypes.c_int, [P, P, i64, P, i64, P, P, P, P, P, P]),
    "idf_rans_decode_on": (ctypes.c_int, [P, P, i64, P, P, i64, i64, P, P, P, P]),
    "idf_rans_encode": (ctypes.c_int, [P, i64, P, P, P, P, P, P]),
    "idf_rans_decode": (ctypes.c_int, [P, P, i64, i64, P, P, P, P]),
    "idf_log_prob": (ctypes.c_int, [P, i64, i64, P, P, P, i32, f32, P, P]),
    "idf_expf_glibc": (ctypes.c_int, [P, i64, P, P]),
    "idf_expf_checksum": (ctypes.c_int, [P, u64, u64, P]),
    "idf_rans_cdf_selfcheck": (ctypes.c_int, [P, u64, u64, P]),
    "idf_rans_part1_selfcheck": (ctypes.c_int, [P, u64, u64, P]),
    "idf_dense_block_f32": (ctypes.c_int, [P, P, i32, i32, i32, P, i64, P, i64, P]),
    "idf_dense_block_dx3_tmp_bytes": (i64, [P, i32, i32, i32]),
    "idf_dx3_block_supported": (ctypes.c_int, [i32, i32, i32, i32]),
    "idf_timer_create": (P, [i32]),
    "idf_timer_destroy": (None, [P]),
    "idf_timer_reset": (None, [P]),
    "idf_timer_summary": (ctypes.c_int, [P, i32, P, P, P]),
    "idf_dense_block_f32_timed": (ctypes.c_int, [P, P, i32, i32, i32, P, i64, P, i64, P, P]),
    "idf_conv1x1_f32": (ctypes.c_int, [P, i64, i32, i32, P, i64, P, i32, i32, P, P, i64, i32, i32,
                                       i32, P]),
    "idf_conv3x3_f32": (ctypes.c_int, [P, i32, i32, i32, i32, P, i64, P, i32, i32, P, i32, P, i64,
                                       i32, f32]),
    "idf_conv3x3_fold_f32": (ctypes.c_int, [P, i32, i32, i32, i32, P, i64, P, i32, i32, P, P, i32,
                                            P, i32, P, i64, i32, f32]),
    "idf_conv3x3_halo_workspace": (i64, [i32, i32, i32, i32, i32]),
    "idf_conv3x3_halo": (ctypes.c_int, [P, i32, i32, i32, i32, P, i64, P, i32, i32, P, P, i32, P,
                                        i32, P, i64, i32, f32, P, i64]),
    "idf_conv3x3_wino_supported": (ctypes.c_int, [i32, i32]),
    "idf_conv3x3_wino_workspace": (i64, [i32, i32, i32, i32, i32]),
    "idf_conv3x3_wino": (ctypes.c_int, [P, i32, i32, i32, i32, P, i64, P, i32, P, P, i32, P, i32, P,
                                        i64, i32, f32, P, i64]),
    "idf_conv3x3_wino_res": (ctypes.c_int, [P, i32, i32, i32, i32, P, i64, P, i32, P, i32, P, i64,
                                            P, i64, i32, f32, P, i64]),
    "idf_conv3x3_wx3": (ctypes.c_int, [P, i32, i32, i32, i32, P, i64, P, i32, f32, P, P, i32, P,
                                       i32, P, i64, i32, f32, P, i32, P, i64]),
    "idf_conv3x3_wx3_res": (ctypes.c_int, [P, i32, i32, i32, i32, P, i64, P, i32, f32, P, i32, P,
                                           i64, P, i64, i32, f32, P, i32, P, i64]),
    "idf_conv3x3_dx3_supported": (ctypes.c_int, [i32, i32, i32]),
    "idf_conv3x3_dx3": (ctypes.c_int, [P, i32, i32, i32, i32, P, i32, P, i32, f32, P, P, i32, P,
                                       i32, P, i64, i32, f32, P, P, i64, P]),
    "idf_dx3_head_init": (ctypes.c_int, [P, i64, i32, P, i64, P, i32, P, i32, P]),
    "idf_conv3x3_dx3_counter_bytes": (i64, [i32, i32, i32, i32]),
    "idf_conv3x3_dx3_workspace": (i64, [i32, i32, i32, i32, i32]),
    "idf_dx3_split_bytes": (i64, [i64, i32]),
    "idf_dx3_split_cols": (ctypes.c_int, [P, i64, i32, i32, P, i64, P, i32, P, P, i32]),
    "idf_dx3_split_cols_head": (ctypes.c_int, [P, i64, i32, P, i64, P, i32, P, P, i32, P, i32, P,
                                               i32, P]),
    "idf_conv3x3_dxb_supported": (ctypes.c_int, [i32, i32, i32]),
    "idf_conv3x3_dxb": (ctypes.c_int, [P, i32, i32, i32, i32, P, i32, P, i32, P, P, i32, P, i32,
                                       P, i64, i32, f32, P, i64, P]),
    "idf_dxb_bytes": (i64, [i64, i32]),
    "idf_dxb_cols": (ctypes.c_int, [P, i64, i32, i32, P, i64, P, i32, P, i32]),
    "idf_conv3x3_bf16_workspace": (i64, [i32, i32, i32, i32, i32]),
    "idf_conv3x3_bf16": (ctypes.c_int, [P, i32, i32, i32, i32, P, i64, P, i32, P, P, i32, P, i32,
                                        P, i64, P, i64, i32, i32, f32, P, i64]),
    "idf_f32_to_bf16_cols": (ctypes.c_int, [P, i64, i32, i32, P, i64, P, i64]),
    "idf_dequant_u8": (ctypes.c_int, [P, i32, i32, i32, i32, P, P, i64]),
    "idf_quant_u8": (ctypes.c_int, [P, i32, i32, i32, i32, P, i64, P, P]),
    "idf_squeeze": (ctypes.c_int, [P, i32, i32, i32, i32, i32, P, i64, P, i64]),
    "idf_unsqueeze": (ctypes.c_int, [P, i32, i32, i32, i32, i32, P, i64, P, i64]),
    "idf_permute_couple_in": (ctypes.c_int, [P, i64, i32, P, P, i64, P, i64, i32, i32, P, i64]),
    "idf_copy_cols": (ctypes.c_int, [P, i64, i32, i32, P, i64, P, i64]),
    "idf_pm_to_nchw": (ctypes.c_int, [P, i32, i32, i32, i32, P, i64, P]),
    "idf_nchw_to_pm": (ctypes.c_int, [P, i32, i32, i32, i32, P, P, i64]),
    "idf_conv_taps_n_alloc": (ctypes.c_int, [i32]),
    "idf_conv_taps_f32": (ctypes.c_int, [P, i32, i32, i32, i32, P, i64, i32, i32, i32, i32, i32, P,
                                         P, P, i32, i32, P, i32, P, i64, i32, i32, i32, i32, i32,
                                         i32, P, i64, i32, f32]),
    "idf_conv_taps_x3": (ctypes.c_int, [P, i32, i32, i32, i32, P, i64, i32, i32, i32, i32, i32, P,
                                        P, P, i32, i32, f32, P, i32, P, i64, i32, i32, i32, i32,
                                        i32, i32, P, i64, i32, f32, P]),
    "idf_vq_norms": (ctypes.c_int, [P, i32, i32, P, i32, P]),
    "idf_vq_argmin": (ctypes.c_int, [P, i64, i32, P, i64, P, i32, i32, P, P]),
    "idf_vq_argmin_ws": (ctypes.c_int, [P, i64, i32, P, i64, P, i32, i32, P, P, P, i64]),
    "idf_vq_argmin_x3_ws": (ctypes.c_int, [P, i64, i32, P, i64, P, i32, f32, i32, P, P,
                                           P, i64, P]),
    "idf_vq_argmin_workspace_bytes": (i64, [i64, i32]),
    "idf_vq_gather": (ctypes.c_int, [P, i64, i32, P, P, i32, P, i64]),
    "idf_vq_pointwise": (ctypes.c_int, [P, i64, i32, i32, P, i64, P, i64, P, i64]),
    "idf_patch": (ctypes.c_int, [P, i32, i32, i32, i32, i32, i32, i32, P, P]),
    "idf_pad_edge_u8": (ctypes.c_int, [P, i32, i32, i32, i32, i32, i32, P, P]),
    "idf_pack_bits_words": (i64, [i64, i64, i32]),
    "idf_pack_bits": (ctypes.c_int, [P, i64, i64, i32, P, P]),
    "idf_unpack_bits": (ctypes.c_int, [P, i64, i64, i32, P, P]),
}

_lib = None


class IdfError(RuntimeError):
    pass


def lib():
    """Load libidfcodec.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise IdfError(f"libidfcodec.so not built ({LIB_PATH}); run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = ""):
    if rc != IDF_OK:
        raise IdfError(f"{what}: {ERR_NAMES.get(rc, rc)}")


def require_device(t: torch.Tensor, what: str = "tensor"):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise IdfError(f"idfcodec: {what} must be a HIP device tensor (no CPU fallback)")


def new_stream(device=None, priority: int | None = None) -> torch.cuda.ExternalStream:
    """A HIP stream created with hipStreamNonBlocking on `device`, as a torch stream.
    The ImageCodec lanes use these: two torch.cuda.Stream()s were measured NOT to run
    concurrently on MI355X (the second lane's kernels waited ~25 ms for the first's), two
    such streams do (tools/lanes_probe.py).  Lives as long as the process."""
    hip = ctypes.CDLL("libamdhip64.so.7")
    h = ctypes.c_void_p()
    with torch.cuda.device(device):
        if priority is None:
            rc = hip.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(1))
        else:  # hipStreamCreateWithPriority: lower numbers run first
            rc = hip.hipStreamCreateWithPriority(ctypes.byref(h), ctypes.c_uint(1),
                                                 ctypes.c_int(int(priority)))
    if rc != 0:
        raise IdfError(f"hipStreamCreateWithFlags failed ({rc})")
    return torch.cuda.ExternalStream(h.value, device=device)


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()

"""rans.rans -- drop-in for the reference's Cython module (rans/rans.pyx:37-110).

encode(state, n, x_, mean_, scale_) -> (state, list[int])
decode(state, buffer_, n, mean_, scale_) -> (state, list[float])

Same signatures, argument conventions (decode takes the buffer, means and
scales REVERSED and returns the symbols reversed, as trainer.py:317 and
coder.py:36 call it), results and exceptions.  Each call is one stream of the
HIP coder (libidfcodec: idf_rans_encode_streams / idf_rans_decode_streams),
bit-identical to the reference.  There is no CPU path: a GPU is required.
"""
import numpy as np
import torch

from idfcodec import _lib
from idfcodec._lib import check, lib, ptr

__all__ = ["encode", "decode"]


def _as_f32(name, v, n):
    if not isinstance(v, list):
        raise TypeError(f"Argument '{name}' has incorrect type (expected list, got {type(v).__name__})")
    if n > len(v):
        # the reference reads past the end of its vector (undefined behaviour)
        raise IndexError(f"n={n} exceeds len({name})={len(v)}")
    return np.asarray(v[:n], dtype=np.float32)


def _raise_status(st: int):
    if st & _lib.STREAM_SCALE_ZERO:
        raise ZeroDivisionError("float division")
    if st & _lib.STREAM_FREQ_ZERO:
        raise ZeroDivisionError("integer division or modulo by zero")
    if st & _lib.STREAM_NEG_CDF:
        raise OverflowError("can't convert negative value to unsigned PY_LONG_LONG")
    if st & _lib.STREAM_UNDERFLOW:
        raise IndexError("rANS buffer exhausted")


def _dev():
    if not torch.cuda.is_available():
        raise _lib.IdfError("rans.rans: no HIP device visible (the coder has no CPU path)")
    return torch.device("cuda")


def encode(state, n, x_, mean_, scale_):
    """rans.pyx:37-67."""
    state = int(state)
    if not 0 <= state < (1 << 64):
        raise OverflowError("can't convert to unsigned PY_LONG_LONG")
    n = int(n)
    x = _as_f32("x_", x_, max(n, 0))
    mean = _as_f32("mean_", mean_, max(n, 0))
    scale = _as_f32("scale_", scale_, max(n, 0))
    if n <= 0:
        return state, []
    dev = _dev()
    d = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    dx, dm, ds = d(x), d(mean), d(scale)
    off = torch.tensor([0, n], dtype=torch.int64, device=dev)
    init = torch.tensor([np.uint64(state).view(np.int64)], dtype=torch.int64, device=dev)
    final = torch.empty(1, dtype=torch.int64, device=dev)
    words = torch.empty(n, dtype=torch.int32, device=dev)
    nw = torch.empty(1, dtype=torch.int64, device=dev)
    status = torch.empty(1, dtype=torch.int32, device=dev)
    wb = lib().idf_rans_encode_workspace_bytes(n)
    ws = torch.empty(wb, dtype=torch.uint8, device=dev)
    check(lib().idf_rans_encode_streams(_lib.stream_ptr(dev), 1, n, ptr(off), ptr(dx), ptr(dm),
                                        ptr(ds), ptr(init), ptr(final), ptr(words), ptr(nw),
                                        ptr(status), ptr(ws), wb), "rans encode")
    _raise_status(int(status.item()))
    k = int(nw.item())
    st = int(np.int64(final.item()).view(np.uint64))
    return st, words[:k].cpu().numpy().view(np.uint32).tolist()


def decode(state, buffer_, n, mean_, scale_):
    """rans.pyx:69-110 (buffer_, mean_, scale_ reversed; result reversed)."""
    state = int(state)
    if not 0 <= state < (1 << 64):
        raise OverflowError("can't convert to unsigned PY_LONG_LONG")
    if not isinstance(buffer_, list):
        raise TypeError(f"Argument 'buffer_' has incorrect type (expected list, got {type(buffer_).__name__})")
    n = int(n)
    mean = _as_f32("mean_", mean_, max(n, 0))
    scale = _as_f32("scale_", scale_, max(n, 0))
    if n <= 0:
        return state, []
    dev = _dev()
    # natural order for the device coder: words in push order, symbols 0..n-1
    words = np.asarray(buffer_[::-1], dtype=np.uint64).astype(np.uint32).view(np.int32)
    nwords = words.size
    dw = torch.from_numpy(words if nwords else np.zeros(1, np.int32)).to(dev)
    dm = torch.from_numpy(np.ascontiguousarray(mean[::-1])).to(dev)
    ds = torch.from_numpy(np.ascontiguousarray(scale[::-1])).to(dev)
    off = torch.tensor([0, n], dtype=torch.int64, device=dev)
    woff = torch.zeros(1, dtype=torch.int64, device=dev)
    nw = torch.tensor([nwords], dtype=torch.int64, device=dev)
    init = torch.tensor([np.uint64(state).view(np.int64)], dtype=torch.int64, device=dev)
    final = torch.empty(1, dtype=torch.int64, device=dev)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    status = torch.empty(1, dtype=torch.int32, device=dev)
    wb = lib().idf_rans_decode_workspace_bytes(n)
    ws = torch.empty(wb, dtype=torch.uint8, device=dev)
    check(lib().idf_rans_decode_streams(_lib.stream_ptr(dev), 1, n, ptr(off), ptr(woff), ptr(nw),
                                        ptr(dw), ptr(dm), ptr(ds), ptr(init), ptr(final), ptr(out),
                                        ptr(status), ptr(ws), wb), "rans decode")
    _raise_status(int(status.item()))
    st = int(np.int64(final.item()).view(np.uint64))
    return st, out.cpu().numpy()[::-1].astype(np.float64).tolist()

"""oracle/rans_oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes front end of oracle/rans_oracle.c, the plain-C restatement of the
reference rANS coder (/root/reference/rans/rans.pyx:25-110).  Used by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg as the parity checker;
never by the product path.

Also loads the reference's own compiled coder from oracle/_ref (built by
oracle/Makefile from /root/reference/rans/rans.cpp) when it is present.
"""
from __future__ import annotations

import ctypes
import importlib.machinery
import importlib.util
import os
import subprocess
import sysconfig

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "librans_oracle.so")
REF_PATH = os.path.join(HERE, "_ref", "rans" + sysconfig.get_config_var("EXT_SUFFIX"))

ERRORS = {
    1: (ZeroDivisionError, "float division"),
    2: (ZeroDivisionError, "integer division or modulo by zero"),
    3: (OverflowError, "can't convert negative value to unsigned int"),
    4: (IndexError, "rANS word buffer exhausted"),
}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        i64 = ctypes.c_int64
        L.oracle_cdf.argtypes = [ctypes.c_float] * 4 + [P]
        L.oracle_cdf.restype = ctypes.c_int
        L.oracle_cdf_freq.argtypes = [i64, P, P, P, P, P]
        L.oracle_rans_encode.argtypes = [P, i64, P, P, P, P, P]
        L.oracle_rans_decode.argtypes = [P, P, i64, i64, P, P, P]
        L.oracle_encode_streams.argtypes = [i64, P, P, P, P, P, P, P, P, P]
        L.oracle_decode_streams.argtypes = [i64, P, P, P, P, P, P, P, P, P, P]
        L.oracle_expf_many.argtypes = [i64, P, P]
        L.oracle_omp_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _raise(code):
    if code:
        exc, msg = ERRORS.get(code, (RuntimeError, f"oracle error {code}"))
        raise exc(msg)


def f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def cdf(x, mean, scale, lower) -> int:
    err = ctypes.c_int(0)
    v = lib().oracle_cdf(x, mean, scale, lower, ctypes.byref(err))
    _raise(err.value)
    return v


def cdf_freq(x, mean, scale):
    x, mean, scale = f32(x), f32(mean), f32(scale)
    n = x.size
    st = np.empty(n, np.int32)
    fr = np.empty(n, np.int32)
    _raise(lib().oracle_cdf_freq(n, _p(x), _p(mean), _p(scale), _p(st), _p(fr)))
    return st, fr


def encode(state: int, x, mean, scale):
    """One reference encode() call (rans.pyx:37-67). Returns (state, words u32 push order)."""
    x, mean, scale = f32(x), f32(mean), f32(scale)
    n = x.size
    st = ctypes.c_uint64(state)
    words = np.empty(max(n, 1), np.uint32)
    nw = ctypes.c_int64(0)
    _raise(lib().oracle_rans_encode(ctypes.byref(st), n, _p(x), _p(mean), _p(scale), _p(words),
                                    ctypes.byref(nw)))
    return st.value, words[: nw.value].copy()


def decode(state: int, words, n: int, mean, scale):
    """One reference decode() call (rans.pyx:69-110) with the reversals folded in:
    words in push order, mean/scale/result in natural order."""
    words = np.ascontiguousarray(np.asarray(words, dtype=np.uint32))
    mean, scale = f32(mean), f32(scale)
    out = np.empty(n, np.float32)
    st = ctypes.c_uint64(state)
    _raise(lib().oracle_rans_decode(ctypes.byref(st), _p(words), words.size, n, _p(mean),
                                    _p(scale), _p(out)))
    return st.value, out


def encode_streams(sym_off, x, mean, scale, init_state=None):
    """Independent streams k = symbols [sym_off[k], sym_off[k+1]).  Returns
    (final_state u64[n], words u32[total] with stream k at sym_off[k], nwords i64[n], status)."""
    sym_off = np.ascontiguousarray(sym_off, dtype=np.int64)
    x, mean, scale = f32(x), f32(mean), f32(scale)
    ns = sym_off.size - 1
    if init_state is None:
        init_state = np.full(ns, 1 << 32, np.uint64)
    init_state = np.ascontiguousarray(init_state, dtype=np.uint64)
    fs = np.empty(ns, np.uint64)
    words = np.empty(max(int(sym_off[-1]), 1), np.uint32)
    nw = np.empty(ns, np.int64)
    status = np.empty(ns, np.int32)
    lib().oracle_encode_streams(ns, _p(sym_off), _p(x), _p(mean), _p(scale), _p(init_state),
                                _p(fs), _p(words), _p(nw), _p(status))
    return fs, words, nw, status


def decode_streams(sym_off, word_off, nwords, words, mean, scale, init_state):
    sym_off = np.ascontiguousarray(sym_off, dtype=np.int64)
    word_off = np.ascontiguousarray(word_off, dtype=np.int64)
    nwords = np.ascontiguousarray(nwords, dtype=np.int64)
    words = np.ascontiguousarray(words, dtype=np.uint32)
    mean, scale = f32(mean), f32(scale)
    init_state = np.ascontiguousarray(init_state, dtype=np.uint64)
    ns = sym_off.size - 1
    fs = np.empty(ns, np.uint64)
    out = np.empty(max(int(sym_off[-1]), 1), np.float32)
    status = np.empty(ns, np.int32)
    lib().oracle_decode_streams(ns, _p(sym_off), _p(word_off), _p(nwords), _p(words), _p(mean),
                                _p(scale), _p(init_state), _p(fs), _p(out), _p(status))
    return fs, out[: int(sym_off[-1])], status


def expf_many(xs):
    xs = f32(xs)
    out = np.empty_like(xs)
    lib().oracle_expf_many(xs.size, _p(xs), _p(out))
    return out


def omp_threads() -> int:
    return int(lib().oracle_omp_threads())


def load_reference_coder():
    """The reference's own Cython coder compiled from rans.cpp (oracle/_ref), or None.
    Loaded under its own name without touching sys.modules['rans']."""
    if not os.path.exists(REF_PATH):
        return None
    loader = importlib.machinery.ExtensionFileLoader("rans", REF_PATH)
    spec = importlib.util.spec_from_file_location("rans", REF_PATH, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod

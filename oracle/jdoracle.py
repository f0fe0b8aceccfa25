"""ctypes binding to the CPU restatement (oracle/out/libjdoracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product.  Parity status:
partially pinned (see jdoracle.h / DESIGN.md "Oracle").
"""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "out", "libjdoracle.so")
_L = None

c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_szp = ctypes.POINTER(ctypes.c_size_t)


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.jdo_deflate.restype = ctypes.c_size_t
        L.jdo_deflate.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint,
                                  ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
        L.jdo_deflate_dict.restype = ctypes.c_size_t
        L.jdo_deflate_dict.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                       ctypes.c_size_t, ctypes.c_int, ctypes.c_uint,
                                       ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
        L.jdo_deflate_calls.restype = ctypes.c_size_t
        L.jdo_deflate_calls.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                        c_szp, ctypes.POINTER(ctypes.c_int), ctypes.c_size_t,
                                        ctypes.c_int, ctypes.c_uint, ctypes.c_void_p,
                                        ctypes.c_size_t]
        L.jdo_deflate_blocks.restype = ctypes.c_size_t
        L.jdo_deflate_blocks.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                         ctypes.c_int, ctypes.c_uint, ctypes.c_void_p,
                                         ctypes.c_size_t, c_u32p]
        L.jdo_bound.restype = ctypes.c_size_t
        L.jdo_bound.argtypes = [ctypes.c_size_t]
        L.jdo_trace.restype = ctypes.c_size_t
        L.jdo_trace.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint,
                                c_u32p, ctypes.c_size_t]
        L.jdo_inflate.restype = ctypes.c_int
        L.jdo_inflate.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                  ctypes.c_size_t, c_szp, c_szp, ctypes.POINTER(ctypes.c_int)]
        L.jdo_inflate_blocks.restype = ctypes.c_int
        L.jdo_inflate_blocks.argtypes = [ctypes.c_void_p, c_u32p, ctypes.c_size_t,
                                         ctypes.c_size_t, ctypes.c_void_p, c_u32p, c_i32p]
        L.jdo_deflate_blocks_mt.restype = ctypes.c_size_t
        L.jdo_deflate_blocks_mt.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                            ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                            c_u32p, ctypes.c_int]
        L.jdo_inflate_blocks_mt.restype = ctypes.c_int
        L.jdo_inflate_blocks_mt.argtypes = [ctypes.c_void_p, c_u64p, c_u32p, ctypes.c_size_t,
                                            ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
        _L = L
    return _L


def _buf(data):
    b = bytes(data)
    return ctypes.create_string_buffer(b, len(b) or 1), len(b)


def deflate(data, level=6, flags=0, flush=1) -> bytes:
    """Fresh reference deflator, whole input, DEFLT_END (1) or DEFLT_FLUSH (2)."""
    src, n = _buf(data)
    cap = lib().jdo_bound(n) + 1024
    out = ctypes.create_string_buffer(cap)
    r = lib().jdo_deflate(src, n, level, flags, flush, out, cap)
    if r == ctypes.c_size_t(-1).value:
        raise RuntimeError("jdo_deflate failed")
    return out.raw[:r]


def deflate_dict(dictionary, data, level=6, flags=0, flush=1) -> bytes:
    """deflator_setdctnr(dictionary) on a fresh deflator, then as deflate()."""
    dct, dn = _buf(dictionary)
    src, n = _buf(data)
    cap = lib().jdo_bound(n) + 1024
    out = ctypes.create_string_buffer(cap)
    r = lib().jdo_deflate_dict(dct, dn, src, n, level, flags, flush, out, cap)
    if r == ctypes.c_size_t(-1).value:
        raise RuntimeError("jdo_deflate_dict failed")
    return out.raw[:r]


def deflate_calls(data, calls, level=6, flags=0, dictionary=b"") -> bytes:
    """A sequence of deflator_deflate calls on one single-window deflator:
    calls = [(end, flush), ...] hands data[prev_end:end] with flush 0
    (NOFLUSH), 2 (DEFLT_FLUSH) or 1 (DEFLT_END); outputs concatenated."""
    src, n = _buf(data)
    dct, dn = _buf(dictionary)
    k = len(calls)
    ends = (ctypes.c_size_t * max(k, 1))(*[e for e, _ in calls])
    fl = (ctypes.c_int * max(k, 1))(*[f for _, f in calls])
    nflush = sum(1 for _, f in calls if f) + 1
    cap = lib().jdo_bound(n) + 1024 + 16 * nflush
    out = ctypes.create_string_buffer(cap)
    r = lib().jdo_deflate_calls(dct if dn else None, dn, src, ends, fl, k, level, flags, out, cap)
    if r == ctypes.c_size_t(-1).value:
        raise RuntimeError("jdo_deflate_calls failed")
    return out.raw[:r]


def deflate_blocks(data, level=6, blocksize=65536, flags=0):
    src, n = _buf(data)
    nb = max(1, -(-n // blocksize))
    cap = nb * (lib().jdo_bound(blocksize) + 1024)
    out = ctypes.create_string_buffer(cap)
    sizes = (ctypes.c_uint32 * nb)()
    r = lib().jdo_deflate_blocks(src, n, blocksize, level, flags, out, cap, sizes)
    if r == ctypes.c_size_t(-1).value:
        raise RuntimeError("jdo_deflate_blocks failed")
    return out.raw[:r], list(sizes)


def trace(data, level=6, flags=0):
    src, n = _buf(data)
    cap = n + 1024
    buf = (ctypes.c_uint32 * cap)()
    k = lib().jdo_trace(src, n, level, flags, buf, cap)
    return list(buf[:k])


def inflate(data, cap):
    """-> (result, error, output, consumed) with inflator.h codes."""
    src, n = _buf(data)
    out = ctypes.create_string_buffer(max(cap, 1))
    cons, prod, err = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_int()
    r = lib().jdo_inflate(src, n, out, cap, ctypes.byref(cons), ctypes.byref(prod),
                          ctypes.byref(err))
    return r, err.value, out.raw[:prod.value], cons.value


def inflate_call(data, n, cap, final):
    """The reference's inflator_inflate after the first n bytes of `data`
    were supplied (inflator.c:765-903): it decodes as far as those bytes
    allow, so its output is the one-shot decode of the prefix, stopped at the
    input end.  -> (result, error, output, consumed):
      the final block ended      -> OK, consumed = bytes up to its last bit
      the input ran out, final=0 -> SRCEXHSTD (:812-815, :849-850), all consumed
      the input ran out, final=1 -> ERROR, EINPUTEND (:806-808, :845-847)
      corrupt data               -> ERROR with its code"""
    r, err, out, cons = inflate(bytes(data[:n]), cap)
    if r == 0:
        return 0, 0, out, cons
    if err == 6 and not final:
        return 1, 0, out, n
    return r, err, out, cons


def inflate_blocks(stream, sizes, blocksize=65536):
    src, n = _buf(stream)
    nb = len(sizes)
    cs = (ctypes.c_uint32 * nb)(*sizes)
    us = (ctypes.c_uint32 * nb)()
    er = (ctypes.c_int32 * nb)()
    out = ctypes.create_string_buffer(nb * blocksize)
    lib().jdo_inflate_blocks(src, cs, nb, blocksize, out, us, er)
    raw = out.raw
    return b"".join(raw[i * blocksize:i * blocksize + us[i]] for i in range(nb)), list(us), list(er)

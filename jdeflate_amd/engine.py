"""ctypes bindings to the MI355X engine (``lib/libjdeflate_amd.so``).

Python mirror of the reference's C interface for the hot path:

* ``Deflator`` / ``Inflator`` drive ``deflator_*`` / ``inflator_*``
  (jdeflate/deflator.h:106-153, inflator.h:97-139) through the C ABI.  The
  header-inline helpers (``deflator_setsrc`` ... ``deflator_tgtend``,
  deflator.h:159-203) write the public struct fields, so they are mirrored
  here on a ctypes copy of that struct (the struct layout is the ABI).
* ``deflate_blocks`` / ``inflate_blocks`` / ``*_device`` wrap the additive
  independent-block batch API (jdeflate/jdgpu.h).

There is no CPU fallback: every entry point raises ``EngineUnavailable``
when the library or a gfx950 device is missing.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(_HERE, "lib")
LIBPATH = os.environ.get("JDAMD_LIB") or os.path.join(LIBDIR, "libjdeflate_amd.so")   # override: dev A/B builds
CORPUSPATH = os.path.join(LIBDIR, "libjdcorpus.so")

# deflator.h:48-76 / inflator.h:48-66
DEFLT_OK, DEFLT_SRCEXHSTD, DEFLT_TGTEXHSTD, DEFLT_ERROR = 0, 1, 2, 3
DEFLT_NOFLUSH, DEFLT_END, DEFLT_FLUSH = 0, 1, 2
DEFLT_SINGLEWINDOW = 0x100       # deflator.h extension: one window over the input
DEFLT_EBADSTATE, DEFLT_EOOM, DEFLT_ELEVEL, DEFLT_EINCORRECTUSE = 1, 2, 3, 4
DEFLT_FIXEDCODES = 1
INFLT_OK, INFLT_SRCEXHSTD, INFLT_TGTEXHSTD, INFLT_ERROR = 0, 1, 2, 3
(INFLT_EBADSTATE, INFLT_EBADCODE, INFLT_EBADTREE, INFLT_EFAROFFSET,
 INFLT_EBADBLOCK, INFLT_EINPUTEND, INFLT_EOOM, INFLT_EINCORRECTUSE) = range(1, 9)

JDGPU_EINVAL, JDGPU_ENODEV, JDGPU_EOOM, JDGPU_ECAP, JDGPU_EDATA = -1, -2, -3, -4, -5
BLOCKSIZE = 65536

# every symbol the C ABI exports (include/jdeflate/*.h)
EXPORTS = (
    "deflator_create", "deflator_destroy", "deflator_reset", "deflator_deflate",
    "deflator_setdctnr", "inflator_create", "inflator_destroy", "inflator_reset",
    "inflator_inflate", "inflator_setdctnr", "jdeflate_getversion",
    "jdgpu_available", "jdgpu_bound", "jdgpu_deflate_device", "jdgpu_inflate_device",
    "jdgpu_deflate", "jdgpu_inflate", "jdgpu_inflate_stream", "jdgpu_prof_enable",
    "jdgpu_prof_read", "jdgpu_debug_deflate", "jdgpu_checksum", "jdgpu_checksum_device",
    "jdgpu_deflate_cs", "jdgpu_inflate_stream_cs", "jdgpu_inflate_flushed",
    "jdgpu_stream_bound", "jdgpu_deflate_stream_device", "jdgpu_deflate_stream",
    "jdgpu_deflate_stream_dict", "jdgpu_inflate_stream_dict", "jdgpu_inflate_resume",
    "jdgpu_stream_create", "jdgpu_stream_deflate", "jdgpu_stream_destroy",
    "jdgpu_istream_create", "jdgpu_istream_reset", "jdgpu_istream_inflate",
    "jdgpu_istream_stats", "jdgpu_istream_fsp", "jdgpu_istream_rpar", "jdgpu_istream_queue",
    "jdgpu_istream_destroy", "jdgpu_deflate_multi", "jdgpu_deflate_multi_device",
    "jdgpu_inflate_multi",
    "zstrm_create", "zstrm_destroy", "zstrm_setsource", "zstrm_setsourcefn",
    "zstrm_settargetfn", "zstrm_setdctnr", "zstrm_inflate", "zstrm_deflate", "zstrm_flush",
    "zstrm_reset", "zstrm_crc32combine", "zstrm_crc32update", "zstrm_adler32update",
)

# zstrm.h:37-90
ZSTRM_INFLATE, ZSTRM_DEFLATE = 0x00010000, 0x00020000
ZSTRM_DFLT, ZSTRM_ZLIB, ZSTRM_GZIP = 0x00100000, 0x00200000, 0x00400000
ZSTRM_DOCRC, ZSTRM_DOADLER, ZSTRM_NOCRC, ZSTRM_NOADLER = 0x01000000, 0x02000000, 0x04000000, 0x08000000
(ZSTRM_OK, ZSTRM_EIOERROR, ZSTRM_EOOM, ZSTRM_EBADDATA, ZSTRM_ECHECKSUM, ZSTRM_EFORMAT,
 ZSTRM_EMISSINGDICT, ZSTRM_ESRCEXHSTD, ZSTRM_ETGTEXHSTD, ZSTRM_EDEFLATE, ZSTRM_EBADDICT,
 ZSTRM_ELIMIT, ZSTRM_EINCORRECTUSE) = range(13)
KERNELS = ("k_chains<4>", "k_chains<3>", "k_match", "k_parse", "k_emit", "k_stored",
           "k_scan", "k_compact", "k_inflate", "k_inflate_par", "k_inflate_resolve",
           "k_pspec", "k_psync", "k_pjoin", "k_checksum", "k_inflate_mp",
           "k_fsp_find", "k_fsp_decode", "k_fsp_window", "k_fsp_resolve", "k_inflate_rpar",
           "k_porder")


class _ZPublic(ctypes.Structure):
    """struct TZStrm (zstrm.h:104-130)."""
    _fields_ = [
        ("state", ctypes.c_uint32), ("error", ctypes.c_uint32), ("flags", ctypes.c_uint32),
        ("smode", ctypes.c_uint32), ("stype", ctypes.c_uint32), ("level", ctypes.c_int32),
        ("total", ctypes.c_size_t), ("dictid", ctypes.c_uint32), ("dict", ctypes.c_uint32),
        ("crc", ctypes.c_uint32), ("adler", ctypes.c_uint32), ("usedinput", ctypes.c_size_t),
    ]


class InflateResult(ctypes.Structure):
    """JDGPUInflateResult (jdeflate/jdgpu.h)."""
    _fields_ = [
        ("produced", ctypes.c_uint64), ("consumed", ctypes.c_uint64),
        ("resumebit", ctypes.c_uint64), ("resumeout", ctypes.c_uint64),
        ("error", ctypes.c_int32), ("parallel", ctypes.c_uint32),
    ]


class InflateStep(ctypes.Structure):
    """JDGPUInflateStep (jdeflate/jdgpu.h)."""
    _fields_ = [
        ("produced", ctypes.c_uint64), ("consumed", ctypes.c_uint64),
        ("status", ctypes.c_int32), ("error", ctypes.c_int32),
        ("parallel", ctypes.c_uint32), ("pad", ctypes.c_uint32),
    ]


IS_ENDED, IS_NEEDINPUT, IS_FULL, IS_ERROR = 0, 1, 2, 3


ZSTRM_IFN = ctypes.CFUNCTYPE(ctypes.c_ssize_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)
ZSTRM_OFN = ctypes.CFUNCTYPE(ctypes.c_ssize_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)


class EngineUnavailable(RuntimeError):
    """The HIP engine (library or gfx950 device) is not usable."""


class _Public(ctypes.Structure):
    """struct TDeflator / struct TInflator (deflator.h:81-99, inflator.h:71-89)."""
    _fields_ = [
        ("state", ctypes.c_uint32), ("error", ctypes.c_uint32),
        ("flags", ctypes.c_uint32), ("flush", ctypes.c_uint32),
        ("status", ctypes.c_uint32),
        ("source", ctypes.c_void_p), ("sbgn", ctypes.c_void_p), ("send", ctypes.c_void_p),
        ("target", ctypes.c_void_p), ("tbgn", ctypes.c_void_p), ("tend", ctypes.c_void_p),
    ]


_lib = None
_corpus = None

c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)


def _init_torch_first() -> None:
    """PyTorch ships its own HIP runtime (ROCm 7.0, no SONAME) next to the
    system one this library links (ROCm 7.2).  Both can live in one process,
    but torch only initialises if its runtime comes up first, so a process
    that uses both brings torch up before loading the engine."""
    try:
        import torch
    except ImportError:
        return
    try:
        if torch.cuda.device_count() > 0:
            torch.cuda.init()
    except Exception:
        pass


def load_library(path: str = LIBPATH) -> ctypes.CDLL:
    """Load the C-ABI library and declare its signatures (no GPU needed)."""
    global _lib
    if _lib is not None:
        return _lib
    _init_torch_first()
    if not os.path.exists(path):
        raise EngineUnavailable(f"{path} not built (run __graft_entry__.build())")
    L = ctypes.CDLL(path)
    P = ctypes.POINTER(_Public)
    L.deflator_create.restype = P
    L.deflator_create.argtypes = [ctypes.c_size_t, ctypes.c_ssize_t, ctypes.c_void_p]
    L.deflator_destroy.argtypes = [P]
    L.deflator_reset.argtypes = [P]
    L.deflator_deflate.restype = ctypes.c_int
    L.deflator_deflate.argtypes = [P, ctypes.c_int]
    L.deflator_setdctnr.argtypes = [P, ctypes.c_void_p, ctypes.c_size_t]
    L.inflator_create.restype = P
    L.inflator_create.argtypes = [ctypes.c_size_t, ctypes.c_void_p]
    L.inflator_destroy.argtypes = [P]
    L.inflator_reset.argtypes = [P]
    L.inflator_inflate.restype = ctypes.c_int
    L.inflator_inflate.argtypes = [P, ctypes.c_uint32]
    L.inflator_setdctnr.argtypes = [P, ctypes.c_void_p, ctypes.c_size_t]
    L.jdgpu_available.restype = ctypes.c_int
    L.jdgpu_bound.restype = ctypes.c_uint64
    L.jdgpu_bound.argtypes = [ctypes.c_uint64, ctypes.c_uint32]
    L.jdgpu_deflate_device.restype = ctypes.c_int
    L.jdgpu_deflate_device.argtypes = [
        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32,
        ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p]
    L.jdgpu_inflate_device.restype = ctypes.c_int
    L.jdgpu_inflate_device.argtypes = [
        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    c_ip = ctypes.POINTER(ctypes.c_int)
    L.jdgpu_deflate_multi.restype = ctypes.c_int64
    L.jdgpu_deflate_multi.argtypes = [
        ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32,
        ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, c_u32p, ctypes.c_int, c_ip]
    L.jdgpu_deflate_multi_device.restype = ctypes.c_int
    L.jdgpu_deflate_multi_device.argtypes = [
        ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32,
        ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), c_u32p,
        ctypes.c_int, c_ip]
    L.jdgpu_inflate_multi.restype = ctypes.c_int
    L.jdgpu_inflate_multi.argtypes = [
        ctypes.c_char_p, ctypes.c_uint64, c_u32p, ctypes.c_uint32, ctypes.c_uint32,
        ctypes.c_void_p, c_u32p, c_i32p, ctypes.c_int, c_ip]
    L.jdgpu_deflate.restype = ctypes.c_int64
    L.jdgpu_deflate.argtypes = [
        ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32,
        ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, c_u32p]
    L.jdgpu_stream_bound.restype = ctypes.c_uint64
    L.jdgpu_stream_bound.argtypes = [ctypes.c_uint64]
    L.jdgpu_deflate_stream.restype = ctypes.c_int64
    L.jdgpu_deflate_stream.argtypes = [
        ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, ctypes.c_int,
        ctypes.c_void_p, ctypes.c_uint64]
    if hasattr(L, "jdgpu_stream_create"):          # (dev A/B builds may predate it)
        L.jdgpu_stream_create.restype = ctypes.c_void_p
        L.jdgpu_stream_create.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint64]
        L.jdgpu_stream_deflate.restype = ctypes.c_int64
        L.jdgpu_stream_deflate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64, c_u64p,
                                           ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64]
        L.jdgpu_stream_destroy.argtypes = [ctypes.c_void_p]
    L.jdgpu_deflate_stream_dict.restype = ctypes.c_int64
    L.jdgpu_deflate_stream_dict.argtypes = [
        ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int,
        ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64]
    L.jdgpu_deflate_stream_device.restype = ctypes.c_int
    L.jdgpu_deflate_stream_device.argtypes = [
        ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32,
        ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    L.jdgpu_inflate.restype = ctypes.c_int
    L.jdgpu_inflate.argtypes = [
        ctypes.c_char_p, ctypes.c_uint64, c_u32p, ctypes.c_uint32, ctypes.c_uint32,
        ctypes.c_void_p, c_u32p, c_i32p]
    L.jdgpu_inflate_stream.restype = ctypes.c_int
    L.jdgpu_inflate_stream.argtypes = [
        ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, c_u64p, c_u64p,
        c_i32p]
    L.jdgpu_prof_enable.restype = ctypes.c_int
    L.jdgpu_prof_enable.argtypes = [ctypes.c_int]
    L.jdgpu_prof_read.restype = ctypes.c_int
    L.jdgpu_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.jdgpu_debug_deflate.restype = ctypes.c_int
    L.jdgpu_debug_deflate.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p]
    L.jdgpu_checksum.restype = ctypes.c_int
    L.jdgpu_checksum.argtypes = [ctypes.c_char_p, ctypes.c_uint64, c_u32p, c_u32p]
    L.jdgpu_checksum_device.restype = ctypes.c_int
    L.jdgpu_checksum_device.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                        ctypes.c_void_p, ctypes.c_void_p]
    L.jdgpu_deflate_cs.restype = ctypes.c_int64
    L.jdgpu_deflate_cs.argtypes = [
        ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32,
        ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, c_u32p, c_u32p, c_u32p]
    L.jdgpu_inflate_flushed.restype = ctypes.c_int
    L.jdgpu_inflate_flushed.argtypes = [
        ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
        c_u64p, c_u64p, c_i32p, c_u32p, c_u32p]
    L.jdgpu_inflate_stream_cs.restype = ctypes.c_int
    L.jdgpu_inflate_stream_cs.argtypes = [
        ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, c_u64p, c_u64p,
        c_i32p, c_u32p, c_u32p]
    L.jdgpu_inflate_resume.restype = ctypes.c_int
    L.jdgpu_inflate_resume.argtypes = [
        ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64,
        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(InflateResult),
        ctypes.c_uint64, c_u32p, c_u32p]
    L.jdgpu_istream_create.restype = ctypes.c_void_p
    L.jdgpu_istream_create.argtypes = []
    L.jdgpu_istream_reset.restype = ctypes.c_int
    L.jdgpu_istream_reset.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64]
    L.jdgpu_istream_inflate.restype = ctypes.c_int
    L.jdgpu_istream_inflate.argtypes = [
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
        ctypes.POINTER(InflateStep), c_u32p, c_u32p]
    L.jdgpu_istream_stats.restype = ctypes.c_int
    L.jdgpu_istream_stats.argtypes = [ctypes.c_void_p, c_u64p, c_u64p, c_u64p]
    L.jdgpu_istream_fsp.restype = ctypes.c_int
    L.jdgpu_istream_fsp.argtypes = [ctypes.c_void_p, ctypes.c_int, c_u64p, c_u64p]
    L.jdgpu_istream_rpar.restype = ctypes.c_int
    L.jdgpu_istream_rpar.argtypes = [ctypes.c_void_p, ctypes.c_int, c_u64p]
    L.jdgpu_istream_queue.restype = ctypes.c_int
    L.jdgpu_istream_queue.argtypes = [ctypes.c_void_p]
    L.jdgpu_istream_destroy.restype = None
    L.jdgpu_istream_destroy.argtypes = [ctypes.c_void_p]
    ZP = ctypes.POINTER(_ZPublic)
    L.zstrm_create.restype = ZP
    L.zstrm_create.argtypes = [ctypes.c_size_t, ctypes.c_ssize_t, ctypes.c_void_p]
    L.zstrm_destroy.argtypes = [ZP]
    L.zstrm_reset.argtypes = [ZP]
    L.zstrm_setsource.argtypes = [ZP, ctypes.c_void_p, ctypes.c_size_t]
    L.zstrm_setsourcefn.argtypes = [ZP, ZSTRM_IFN, ctypes.c_void_p]
    L.zstrm_settargetfn.argtypes = [ZP, ZSTRM_OFN, ctypes.c_void_p]
    L.zstrm_setdctnr.argtypes = [ZP, ctypes.c_void_p, ctypes.c_size_t]
    L.zstrm_inflate.restype = ctypes.c_size_t
    L.zstrm_inflate.argtypes = [ZP, ctypes.c_void_p, ctypes.c_size_t]
    L.zstrm_deflate.restype = ctypes.c_size_t
    L.zstrm_deflate.argtypes = [ZP, ctypes.c_void_p, ctypes.c_size_t]
    L.zstrm_flush.argtypes = [ZP, ctypes.c_uint32]
    L.zstrm_crc32combine.restype = ctypes.c_uint32
    L.zstrm_crc32combine.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t]
    L.zstrm_crc32update.restype = ctypes.c_uint32
    L.zstrm_crc32update.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
    L.zstrm_adler32update.restype = ctypes.c_uint32
    L.zstrm_adler32update.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
    _lib = L
    return L


def prof_enable(on: bool = True) -> None:
    """Per-kernel HIP-event timing on/off (resets totals)."""
    if load_library().jdgpu_prof_enable(1 if on else 0):
        raise RuntimeError("jdgpu_prof_enable failed")


def prof_read() -> dict:
    """{kernel: (total_ms, launches)} since prof_enable."""
    ms = (ctypes.c_double * 32)()
    cnt = (ctypes.c_uint64 * 32)()
    k = load_library().jdgpu_prof_read(ms, cnt, 32)
    return {KERNELS[i]: (ms[i], cnt[i]) for i in range(min(k, len(KERNELS))) if cnt[i]}


def available() -> bool:
    try:
        return bool(load_library().jdgpu_available())
    except (EngineUnavailable, OSError):
        return False


def _need():
    L = load_library()
    if not L.jdgpu_available():
        raise EngineUnavailable("no gfx950 device visible to the HIP runtime")
    return L


def bound(n: int, blocksize: int = BLOCKSIZE) -> int:
    return int(load_library().jdgpu_bound(n, blocksize))


def nblocks(n: int, blocksize: int = BLOCKSIZE) -> int:
    return max(1, -(-n // blocksize))


def deflate_blocks(data: bytes, level: int = 6, blocksize: int = BLOCKSIZE,
                   flags: int = 0, lastflush: int = DEFLT_END):
    """Independent-block deflate on the GPU; returns (stream, per-block sizes)."""
    L = _need()
    nb = nblocks(len(data), blocksize)
    cap = bound(len(data), blocksize)
    out = ctypes.create_string_buffer(cap)
    sizes = (ctypes.c_uint32 * nb)()
    r = L.jdgpu_deflate(bytes(data), len(data), blocksize, level, flags, lastflush,
                        out, cap, sizes)
    if r < 0:
        raise RuntimeError(f"jdgpu_deflate failed: {r}")
    return out.raw[:r], list(sizes)


def _devlist(devices):
    if not devices:
        return 0, None
    return len(devices), (ctypes.c_int * len(devices))(*devices)


def deflate_multi(data: bytes, level: int = 6, blocksize: int = BLOCKSIZE, flags: int = 0,
                  lastflush: int = DEFLT_END, devices=None):
    """jdgpu_deflate_multi: contiguous block ranges over several devices (all
    visible ones when `devices` is None), gathered to the first over RCCL;
    returns (stream, per-block sizes)."""
    L = _need()
    nb = nblocks(len(data), blocksize)
    cap = bound(len(data), blocksize)
    out = ctypes.create_string_buffer(cap)
    sizes = (ctypes.c_uint32 * nb)()
    nd, dv = _devlist(devices)
    r = L.jdgpu_deflate_multi(bytes(data), len(data), blocksize, level, flags, lastflush,
                              out, cap, sizes, nd, dv)
    if r < 0:
        raise RuntimeError(f"jdgpu_deflate_multi failed: {r}")
    return out.raw[:r], list(sizes)


def inflate_multi(stream: bytes, sizes, blocksize: int = BLOCKSIZE, devices=None):
    """jdgpu_inflate_multi; returns (bytes, usizes, errors)."""
    L = _need()
    nb = len(sizes)
    cs = (ctypes.c_uint32 * nb)(*sizes)
    us = (ctypes.c_uint32 * nb)()
    er = (ctypes.c_int32 * nb)()
    out = ctypes.create_string_buffer(nb * blocksize)
    nd, dv = _devlist(devices)
    r = L.jdgpu_inflate_multi(bytes(stream), len(stream), cs, nb, blocksize, out, us, er, nd, dv)
    if r < 0 and r != -5:
        raise RuntimeError(f"jdgpu_inflate_multi failed: {r}")
    raw = out.raw
    return (b"".join(raw[i * blocksize:i * blocksize + us[i]] for i in range(nb)),
            list(us), list(er))


def deflate_stream(data: bytes, level: int = 6, flags: int = 0, flush: int = DEFLT_END,
                   dictionary: bytes = b"") -> bytes:
    """Single-window stream deflate on the GPU: the reference's output for the
    whole input given at once (after deflator_setdctnr(dictionary) when one is
    given) and driven with `flush`."""
    L = _need()
    cap = int(L.jdgpu_stream_bound(len(data)))
    out = ctypes.create_string_buffer(cap + 1)
    dct = bytes(dictionary)
    r = L.jdgpu_deflate_stream_dict(dct or b"\0", len(dct), bytes(data), len(data), level, flags,
                                    flush, out, cap)
    if r < 0:
        raise RuntimeError(f"jdgpu_deflate_stream failed: {r}")
    return out.raw[:r]


def inflate_blocks(stream: bytes, sizes, blocksize: int = BLOCKSIZE):
    """Independent-block inflate on the GPU; returns (data, usizes, errors)."""
    L = _need()
    nb = len(sizes)
    cs = (ctypes.c_uint32 * nb)(*sizes)
    us = (ctypes.c_uint32 * nb)()
    er = (ctypes.c_int32 * nb)()
    out = ctypes.create_string_buffer(nb * blocksize)
    r = L.jdgpu_inflate(bytes(stream), len(stream), cs, nb, blocksize, out, us, er)
    if r < 0 and r != JDGPU_EDATA:
        raise RuntimeError(f"jdgpu_inflate failed: {r}")
    raw = out.raw
    data = b"".join(raw[i * blocksize:i * blocksize + us[i]] for i in range(nb))
    return data, list(us), list(er)


def inflate_stream(stream: bytes, cap: int):
    """Single-stream inflate on the GPU; returns (data, error, consumed)."""
    L = _need()
    out = ctypes.create_string_buffer(max(cap, 1))
    prod = ctypes.c_uint64()
    used = ctypes.c_uint64()
    err = ctypes.c_int32()
    r = L.jdgpu_inflate_stream(bytes(stream), len(stream), out, cap, ctypes.byref(prod),
                               ctypes.byref(used), ctypes.byref(err))
    if r < 0:
        raise RuntimeError(f"jdgpu_inflate_stream failed: {r}")
    return out.raw[:prod.value], err.value, used.value


def deflate_device(d_in: int, n: int, d_out: int, outcap: int, d_csizes: int,
                   d_coffs: int, d_total: int, level: int = 6,
                   blocksize: int = BLOCKSIZE, flags: int = 0,
                   lastflush: int = DEFLT_END, stream: int = 0) -> None:
    """Asynchronous device-resident deflate (pointers are device addresses)."""
    r = load_library().jdgpu_deflate_device(d_in, n, blocksize, level, flags, lastflush,
                                            d_out, outcap, d_csizes, d_coffs, d_total,
                                            stream or None)
    if r:
        raise RuntimeError(f"jdgpu_deflate_device failed: {r}")


def inflate_device(d_in: int, inlen: int, d_coffs: int, d_csizes: int, nb: int,
                   d_out: int, d_usizes: int, d_errors: int,
                   blocksize: int = BLOCKSIZE, stream: int = 0) -> None:
    """Asynchronous device-resident inflate of independent blocks."""
    r = load_library().jdgpu_inflate_device(d_in, inlen, d_coffs, d_csizes, nb, blocksize,
                                            d_out, d_usizes, d_errors, stream or None)
    if r:
        raise RuntimeError(f"jdgpu_inflate_device failed: {r}")


class Deflator:
    """deflator_* through the C ABI, with the header inlines mirrored."""

    def __init__(self, level: int = 6, flags: int = 0):
        L = _need()
        self._L = L
        self._p = L.deflator_create(flags, level, None)
        if not self._p:
            raise ValueError(f"deflator_create(level={level}) returned NULL")
        self._keep = []

    @property
    def public(self) -> _Public:
        return self._p.contents

    def setsrc(self, buf) -> None:           # deflator.h:159-182
        s = self.public
        if s.flush:
            if s.error == 0:
                s.error = DEFLT_EINCORRECTUSE
                s.state = 0xDEADBEEF
            return
        b = ctypes.create_string_buffer(bytes(buf), len(buf))
        self._keep = [b]
        a = ctypes.addressof(b)
        s.source = s.sbgn = a
        s.send = a + len(buf)

    def settgt(self, n: int) -> None:        # deflator.h:184-190
        t = ctypes.create_string_buffer(n)
        self._tgt = t
        a = ctypes.addressof(t)
        s = self.public
        s.target = s.tbgn = a
        s.tend = a + n

    def srcend(self) -> int:
        s = self.public
        return (s.source or 0) - (s.sbgn or 0)

    def tgtend(self) -> int:
        s = self.public
        return (s.target or 0) - (s.tbgn or 0)

    def output(self) -> bytes:
        return self._tgt.raw[:self.tgtend()]

    def deflate(self, flush: int) -> int:
        return self._L.deflator_deflate(self._p, flush)

    def reset(self) -> None:
        self._L.deflator_reset(self._p)

    def close(self) -> None:
        # also reached from __del__ when __init__ failed before _p was set
        if getattr(self, "_p", None):
            self._L.deflator_destroy(self._p)
            self._p = None

    __del__ = close

    def compress(self, data: bytes, chunk: int = 1 << 30, tgt: int = 1 << 20,
                 flush: int = DEFLT_END) -> bytes:
        """The reference's streaming loop (deflator.h:24-36)."""
        out = []
        pos = 0
        while True:
            piece = data[pos:pos + chunk]
            pos += len(piece)
            final = pos >= len(data)
            if piece:
                self.setsrc(piece)
            elif self.public.source is None:
                self.setsrc(b"\0")          # the reference needs a non-NULL source
                self.public.send = self.public.source
            while True:
                self.settgt(tgt)
                r = self.deflate(flush if final else DEFLT_NOFLUSH)
                out.append(self.output())
                if r != DEFLT_TGTEXHSTD:
                    break
            if r != DEFLT_SRCEXHSTD:
                break
        if r != DEFLT_OK:
            raise RuntimeError(f"deflator_deflate -> {r}, error {self.public.error}")
        return b"".join(out)


def deflate_calls(data: bytes, calls, level: int = 6, flags: int = 0, dictionary: bytes = b"",
                  tgt: int = 1 << 20) -> bytes:
    """The drop-in deflator in single-window mode driven with a call sequence
    (oracle deflate_calls' model): calls = [(end, flush), ...] hands
    data[previous end:end] with flush 0, DEFLT_FLUSH or DEFLT_END, draining
    the target between calls; the outputs joined."""
    d = Deflator(level, flags | DEFLT_SINGLEWINDOW)
    keep = None
    if dictionary:
        keep = ctypes.create_string_buffer(bytes(dictionary), len(dictionary))
        d._L.deflator_setdctnr(d._p, keep, len(dictionary))
    out = []
    prev = 0
    try:
        for end, fl in calls:
            piece = data[prev:end]
            prev = end
            if piece:
                d.setsrc(piece)
            else:
                d.setsrc(b"\0")
                d.public.send = d.public.source
            while True:
                d.settgt(tgt)
                r = d.deflate(fl)
                out.append(d.output())
                if r != DEFLT_TGTEXHSTD:
                    break
            if r != (DEFLT_OK if fl else DEFLT_SRCEXHSTD):
                raise RuntimeError(f"deflator_deflate -> {r}, error {d.public.error}")
    finally:
        d.close()
    return b"".join(out)


class Inflator:
    """inflator_* through the C ABI, with the header inlines mirrored."""

    def __init__(self, flags: int = 0):
        L = _need()
        self._L = L
        self._p = L.inflator_create(flags, None)
        if not self._p:
            raise RuntimeError("inflator_create returned NULL")

    @property
    def public(self) -> _Public:
        return self._p.contents

    def setsrc(self, buf) -> None:           # inflator.h:145-168
        s = self.public
        if s.flush:                          # `finalinput` shares the slot
            if s.error == 0:
                s.error = INFLT_EINCORRECTUSE
                s.state = 0xDEADBEEF
            return
        b = ctypes.create_string_buffer(bytes(buf), len(buf))
        self._src = b
        a = ctypes.addressof(b)
        s.source = s.sbgn = a
        s.send = a + len(buf)

    def settgt(self, n: int) -> None:
        t = ctypes.create_string_buffer(n)
        self._tgt = t
        a = ctypes.addressof(t)
        s = self.public
        s.target = s.tbgn = a
        s.tend = a + n

    def tgtend(self) -> int:
        s = self.public
        return (s.target or 0) - (s.tbgn or 0)

    def output(self) -> bytes:
        return self._tgt.raw[:self.tgtend()]

    def inflate(self, final: int) -> int:
        return self._L.inflator_inflate(self._p, final)

    def close(self) -> None:
        # also reached from __del__ when __init__ failed before _p was set
        if getattr(self, "_p", None):
            self._L.inflator_destroy(self._p)
            self._p = None

    __del__ = close

    def srcend(self) -> int:
        s = self.public
        return (s.source or 0) - (s.sbgn or 0)

    def setdctnr(self, d: bytes) -> None:    # inflator.h:129-131
        self._dct = ctypes.create_string_buffer(bytes(d), len(d))
        self._L.inflator_setdctnr(self._p, self._dct, len(d))

    def decompress(self, data: bytes, chunk: int = 1 << 30, tgt: int = 1 << 20,
                   final: str = "last", trace: list | None = None):
        """The reference's streaming loop; returns (bytes, result, error).

        final="last": final=1 with the last chunk; "never": final=0 on every
        call, as zstrm.c:926 in callback mode (the stream's own end returns
        INFLT_OK, inflator.c:829-833).  trace (optional) receives, per call,
        (chunk index, result, bytes delivered so far, bytes of that chunk
        consumed)."""
        out = []
        pos = 0
        got = 0
        r = INFLT_ERROR
        k = 0
        self.consumed = 0
        while True:
            piece = data[pos:pos + chunk]
            pos += len(piece)
            fin = 1 if (final == "last" and pos >= len(data)) else 0
            self.setsrc(piece if piece else b"\0")
            if not piece:
                self.public.send = self.public.source
            while True:
                self.settgt(tgt)
                r = self.inflate(fin)
                o = self.output()
                got += len(o)
                out.append(o)
                if trace is not None:
                    trace.append((k, r, got, self.srcend()))
                if r != INFLT_TGTEXHSTD:
                    break
            self.consumed = pos - len(piece) + self.srcend()
            k += 1
            if r != INFLT_SRCEXHSTD or not piece:
                break
        return b"".join(out), r, self.public.error


class IStream:
    """jdgpu_istream_*: the resumable stream decoder behind the drop-in
    inflator, driven directly (tests and the bench)."""

    def __init__(self, dict_: bytes | None = None):
        L = _need()
        self._L = L
        self._p = L.jdgpu_istream_create()
        if not self._p:
            raise RuntimeError("jdgpu_istream_create returned NULL")
        if dict_:
            if L.jdgpu_istream_reset(self._p, bytes(dict_), len(dict_)):
                raise RuntimeError("jdgpu_istream_reset failed")

    def inflate(self, src, cap: int, src_addr: int | None = None, out=None):
        """-> (status, error, produced, consumed, parallel); output in `out`
        (a ctypes buffer of >= cap bytes, made here when None)"""
        if out is None:
            out = ctypes.create_string_buffer(max(cap, 1))
        self.out = out
        if src_addr is None:
            self._src = ctypes.create_string_buffer(bytes(src), max(len(src), 1))
            src_addr, n = ctypes.addressof(self._src), len(src)
        else:
            n = src
        st = InflateStep()
        r = self._L.jdgpu_istream_inflate(self._p, src_addr, n, out, cap, ctypes.byref(st),
                                          None, None)
        if r:
            raise RuntimeError(f"jdgpu_istream_inflate failed: {r}")
        return st.status, st.error, st.produced, st.consumed, st.parallel

    def stats(self):
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self._L.jdgpu_istream_stats(self._p, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return a.value, b.value, c.value

    def fsp(self, enable: int = -1):
        """parallel decode of marker-free input: enable 1/0 (-1: unchanged);
        -> (rounds, chunks accepted)"""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        self._L.jdgpu_istream_fsp(self._p, enable, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    def rpar(self, enable: int = -1) -> int:
        """the span at hand decoded by 64 lanes: enable 1/0 (-1: unchanged);
        -> its launches so far"""
        a = ctypes.c_uint64()
        self._L.jdgpu_istream_rpar(self._p, enable, ctypes.byref(a))
        return a.value

    def own_queue(self) -> bool:
        """True when the instance has a hardware queue of its own (the first
        16 live instances), False when it shares the process's queues"""
        return self._L.jdgpu_istream_queue(self._p) == 1

    def close(self) -> None:
        if getattr(self, "_p", None):
            self._L.jdgpu_istream_destroy(self._p)
            self._p = None

    __del__ = close


def _corpus_lib():
    global _corpus
    if _corpus is None:
        if not os.path.exists(CORPUSPATH):
            raise EngineUnavailable(f"{CORPUSPATH} not built")
        C = ctypes.CDLL(CORPUSPATH)
        C.jdc_text.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int]
        C.jdc_mixed.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                ctypes.c_uint64, ctypes.c_int]
        _corpus = C
    return _corpus


def corpus_text(n: int, seed: int = 1, threads: int = 8, out=None):
    """English-like Zipf text (config C2); returns a numpy uint8 array."""
    import numpy as np
    a = out if out is not None else np.empty(n, dtype=np.uint8)
    _corpus_lib().jdc_text(a.ctypes.data, n, seed, threads)
    return a


def corpus_mixed(n: int, seed: int = 1, blocksize: int = BLOCKSIZE, threads: int = 8, out=None):
    """Silesia-like per-block mix (config C5); returns a numpy uint8 array."""
    import numpy as np
    a = out if out is not None else np.empty(n, dtype=np.uint8)
    _corpus_lib().jdc_mixed(a.ctypes.data, n, blocksize, seed, threads)
    return a


def checksums(data: bytes, crc: int = 0xFFFFFFFF, adler: int = 1):
    """(CRC-32 register, Adler-32) updated over data on the GPU with the zstrm
    semantics (zstrm_crc32update / zstrm_adler32update): the register is not
    inverted, so a standard CRC-32 is checksums(d)[0] ^ 0xFFFFFFFF."""
    L = _need()
    c = ctypes.c_uint32(crc)
    a = ctypes.c_uint32(adler)
    r = L.jdgpu_checksum(bytes(data), len(data), ctypes.byref(c), ctypes.byref(a))
    if r:
        raise RuntimeError(f"jdgpu_checksum failed: {r}")
    return c.value, a.value


def crc32_combine(crc1: int, crc2: int, len2: int) -> int:
    """zstrm_crc32combine (host algebra, no GPU needed)."""
    return int(load_library().zstrm_crc32combine(crc1, crc2, len2))


class ZStrm:
    """zstrm_* through the C ABI (jdeflate/zstrm.h)."""

    def __init__(self, flags: int, level: int = 6):
        L = _need()
        self._L = L
        self._p = L.zstrm_create(flags, level, None)
        if not self._p:
            raise ValueError(f"zstrm_create({flags:#x}, {level}) failed")
        self._keep = []

    @property
    def public(self) -> _ZPublic:
        return self._p.contents

    def close(self) -> None:
        if getattr(self, "_p", None):
            self._L.zstrm_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # deflate -----------------------------------------------------------------
    def compress(self, data: bytes, chunk: int = 1 << 30, flushes=()):
        """Deflate data in `chunk`-byte zstrm_deflate calls (zstrm_flush(0)
        after the calls listed in flushes), then zstrm_flush(1)."""
        out = []

        def ofn(buf, size, user):
            out.append(ctypes.string_at(buf, size))
            return size
        cb = ZSTRM_OFN(ofn)
        self._keep.append(cb)
        self._L.zstrm_settargetfn(self._p, cb, None)
        src = bytes(data)
        k = 0
        for o in range(0, len(src), chunk):
            piece = src[o:o + chunk]
            n = self._L.zstrm_deflate(self._p, piece, len(piece))
            if n != len(piece):
                break
            if k in flushes:
                self._L.zstrm_flush(self._p, 0)
            k += 1
        self._L.zstrm_flush(self._p, 1)
        return b"".join(out)

    # inflate -----------------------------------------------------------------
    def decompress(self, data: bytes, chunk: int = 1 << 20, callback: bool = False,
                   readsize: int = 32768):
        """Inflate a whole container from a buffer (or through the source
        callback in readsize pieces); zstrm_inflate asked for chunk bytes at a
        time until it returns less.  Returns (bytes, error, state)."""
        src = bytes(data)
        if callback:
            pos = [0]

            def ifn(buf, size, user):
                k = min(size, readsize, len(src) - pos[0])
                ctypes.memmove(buf, src[pos[0]:pos[0] + k], k)
                pos[0] += k
                return k
            cb = ZSTRM_IFN(ifn)
            self._keep.append(cb)
            self._L.zstrm_setsourcefn(self._p, cb, None)
        else:
            self._src = ctypes.create_string_buffer(src, len(src))
            self._L.zstrm_setsource(self._p, self._src, len(src))
        out = []
        buf = ctypes.create_string_buffer(max(chunk, 1))
        while True:
            n = self._L.zstrm_inflate(self._p, buf, chunk)
            out.append(buf.raw[:n])
            if n < chunk:
                break
        return b"".join(out), self.public.error, self.public.state

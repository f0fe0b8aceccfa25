"""The zstrm container (jdeflate/zstrm.h) and the
GPU CRC-32 / Adler-32 scans.

Parity is pinned by independent implementations: Python's zlib (crc32,
adler32, compress/decompress) and gzip, which read every container zstrm
writes and produce every container zstrm reads here.  The reference ships no
test vectors for zstrm; its behaviour is restated from zstrm.c (cited in
jdeflate_amd/csrc/zstrm.c) and the deliberate differences are listed in
include/jdeflate/zstrm.h."""
import ctypes
import gzip
import os
import struct
import zlib

import numpy as np
import pytest

import jdeflate_amd.engine as E

BS = 65536


def _rand(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


# ---- CPU: host algebra and ABI ------------------------------------------------

def test_crc32combine_matches_zlib(built_lib):
    rng = np.random.default_rng(1)
    for la, lb in [(0, 0), (1, 0), (0, 1), (5, 7), (100, 65536), (3, 1 << 20), (70000, 12345)]:
        a = rng.integers(0, 256, la, dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, lb, dtype=np.uint8).tobytes()
        # standard CRCs combine with the same operator (the inversions cancel)
        assert E.crc32_combine(zlib.crc32(a), zlib.crc32(b), lb) == zlib.crc32(a + b)


def test_zstrm_struct_layout():
    assert ctypes.sizeof(E._ZPublic) == 56          # zstrm.h:104-130 on LP64


def test_zstrm_refuses_without_gpu(built_lib):
    import jdeflate_amd as J
    if J.available():
        pytest.skip("GPU present")
    L = J.load_library()
    assert not L.zstrm_create(E.ZSTRM_DEFLATE | E.ZSTRM_GZIP, 6, None)
    assert not L.zstrm_create(E.ZSTRM_INFLATE, 0, None)


def test_zstrm_program_compiles(built_lib, tmp_path):
    prog = tmp_path / "z.c"
    prog.write_text(r'''
#include <jdeflate/zstrm.h>
#include <stdio.h>
int main(void) {
    const TZStrm* z = zstrm_create(ZSTRM_DEFLATE | ZSTRM_GZIP, 6, NULL);
    printf("%d %u\n", (int) sizeof(TZStrm), zstrm_crc32combine(0u, 0u, 5));
    zstrm_destroy(z);
    return 0;
}
''')
    exe = tmp_path / "z"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    import subprocess
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", inc, str(prog), "-o", str(exe),
                    "-L", os.path.dirname(built_lib), "-ljdeflate_amd",
                    "-Wl,-rpath," + os.path.dirname(built_lib)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert out == ["56", "0"]


# ---- GPU: checksum scans -------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 255, 256, 4097, 65535, 65536, 65537,
                               3 * 65536 + 5, (1 << 20) + 3])
def test_checksums_match_zlib(engine, n):
    for d in (_rand(n, n), bytes(n), b"\xff" * n):
        c, a = engine.checksums(d)
        assert c ^ 0xFFFFFFFF == zlib.crc32(d), n
        assert a == zlib.adler32(d), n


@pytest.mark.gpu
def test_checksums_chain_and_large(engine):
    d = engine.corpus_text(300 << 20, seed=3).tobytes()      # > one 256 MiB staging chunk
    c, a = engine.checksums(d)
    assert c ^ 0xFFFFFFFF == zlib.crc32(d) and a == zlib.adler32(d)
    # chained updates from arbitrary running values (zstrm semantics)
    x, y = d[:1000003], d[1000003:3000000]
    c1, a1 = engine.checksums(x)
    c2, a2 = engine.checksums(y, c1, a1)
    assert c2 ^ 0xFFFFFFFF == zlib.crc32(x + y) and a2 == zlib.adler32(x + y)
    L = engine.load_library()
    assert L.zstrm_crc32update(0xFFFFFFFF, y, len(y)) ^ 0xFFFFFFFF == zlib.crc32(y)
    assert L.zstrm_adler32update(1, y, len(y)) == zlib.adler32(y)


@pytest.mark.gpu
def test_checksum_device_blocks(engine):
    import torch
    n = 5 * BS + 777
    host = np.frombuffer(_rand(n, 9), np.uint8)
    d = torch.from_numpy(host.copy()).cuda()
    out = torch.zeros(3 * 6, dtype=torch.int32, device="cuda")
    L = engine.load_library()
    assert L.jdgpu_checksum_device(d.data_ptr(), n, BS, out.data_ptr(), None) == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy().astype(np.uint32).reshape(6, 3)
    for b in range(6):
        blk = host[b * BS:(b + 1) * BS].tobytes()
        # register from 0 = standard CRC of the block with the init/final
        # inversions undone: crc32(blk) ^ crc32(zeros) relation via combine
        ref0 = zlib.crc32(blk) ^ 0xFFFFFFFF
        ref0 ^= E.crc32_combine(0xFFFFFFFF, 0, len(blk))
        assert int(got[b, 0]) == ref0
        x = np.frombuffer(blk, np.uint8).astype(np.uint64)
        w = np.arange(len(blk), 0, -1, dtype=np.uint64)
        assert int(got[b, 1]) == int(x.sum() % 65521)
        assert int(got[b, 2]) == int((x * w).sum() % 65521)


# ---- GPU: zstrm deflate --------------------------------------------------------

def _unpack(kind, c):
    if kind == "gzip":
        return gzip.decompress(c)
    if kind == "zlib":
        return zlib.decompress(c)
    return zlib.decompressobj(-15).decompress(c)


TYPES = {"gzip": E.ZSTRM_GZIP, "zlib": E.ZSTRM_ZLIB, "raw": E.ZSTRM_DFLT}


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["gzip", "zlib", "raw"])
@pytest.mark.parametrize("level", [0, 1, 6, 9])
def test_zstrm_deflate_readable_by_zlib(engine, kind, level):
    for d in (b"", b"x", engine.corpus_text(3 * BS + 11, seed=level).tobytes(),
              engine.corpus_mixed(5 * BS, seed=level).tobytes()):
        z = engine.ZStrm(E.ZSTRM_DEFLATE | TYPES[kind], level)
        c = z.compress(d)
        assert z.public.error == 0 and z.public.state == 4
        assert z.public.total == len(d)
        assert _unpack(kind, c) == d, (kind, level, len(d))
        if kind == "zlib":
            assert c[:2] == b"\x78\x01"               # valid FCHECK (reference: 78 1F)
            assert (c[0] * 256 + c[1]) % 31 == 0


@pytest.mark.gpu
def test_zstrm_deflate_chunks_flushes_and_batches(engine):
    d = engine.corpus_text(40 << 20, seed=5).tobytes()        # > two 16 MiB batches
    for kind in ("gzip", "zlib"):
        z = engine.ZStrm(E.ZSTRM_DEFLATE | TYPES[kind], 6)
        c = z.compress(d, chunk=(3 << 20) + 17, flushes=(2, 5))
        assert _unpack(kind, c) == d
        if kind == "gzip":
            assert z.public.crc == zlib.crc32(d)
        else:
            assert z.public.adler == zlib.adler32(d)
    # raw stream with forced checksums
    z = engine.ZStrm(E.ZSTRM_DEFLATE | E.ZSTRM_DFLT | E.ZSTRM_DOCRC | E.ZSTRM_DOADLER, 6)
    c = z.compress(d[:5 << 20])
    assert _unpack("raw", c) == d[:5 << 20]
    # no trailer: the register is left uninverted (emitgziptail inverts it, zstrm.c:1238)
    assert z.public.crc ^ 0xFFFFFFFF == zlib.crc32(d[:5 << 20])
    assert z.public.adler == zlib.adler32(d[:5 << 20])


@pytest.mark.gpu
def test_zstrm_create_validation(engine):
    L = engine.load_library()
    assert not L.zstrm_create(E.ZSTRM_DEFLATE, 6, None)                      # no type
    assert not L.zstrm_create(E.ZSTRM_DEFLATE | E.ZSTRM_GZIP, 10, None)      # level
    assert not L.zstrm_create(E.ZSTRM_DEFLATE | E.ZSTRM_GZIP | E.ZSTRM_ZLIB, 6, None)
    assert not L.zstrm_create(0, 6, None)                                     # no mode
    z = engine.ZStrm(E.ZSTRM_INFLATE, 0)
    assert z.public.state == 0
    # deflate call on an inflate stream: EINCORRECTUSE, state END
    assert L.zstrm_deflate(z._p, b"abc", 3) == 0
    assert z.public.error == E.ZSTRM_EINCORRECTUSE and z.public.state == 4


# ---- GPU: zstrm inflate --------------------------------------------------------

def _gzip_with_fields(raw_deflate, data, fextra=b"", fname=b"", fcomment=b"", fhcrc=False):
    flg = (0x04 if fextra else 0) | (0x08 if fname else 0) | (0x10 if fcomment else 0) | \
          (0x02 if fhcrc else 0)
    h = b"\x1f\x8b\x08" + bytes([flg]) + b"\x01\x02\x03\x04\x00\x03"
    if fextra:
        h += struct.pack("<H", len(fextra)) + fextra
    if fname:
        h += fname + b"\x00"
    if fcomment:
        h += fcomment + b"\x00"
    if fhcrc:
        h += struct.pack("<H", zlib.crc32(h) & 0xFFFF)
    return h + raw_deflate + struct.pack("<II", zlib.crc32(data), len(data) & 0xFFFFFFFF)


def _raw(data, level=6):
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    return c.compress(data) + c.flush()


@pytest.mark.gpu
@pytest.mark.parametrize("callback", [False, True])
def test_zstrm_inflate_python_containers(engine, callback):
    d = engine.corpus_text(700000, seed=2).tobytes()
    cases = [
        ("gzip", gzip.compress(d, 9), d),
        ("gzip-fields", _gzip_with_fields(_raw(d), d, b"AB\x02\x00xy", b"name.txt", b"hi", True), d),
        ("zlib", zlib.compress(d, 6), d),
        ("zlib1", zlib.compress(d[:1000], 1), d[:1000]),
        ("raw", _raw(d, 9), d),
        ("empty-gzip", gzip.compress(b""), b""),
    ]
    for name, c, want in cases:
        for chunk in (1 << 20, 4096, len(want) or 1):
            z = engine.ZStrm(E.ZSTRM_INFLATE, 0)
            got, err, state = z.decompress(c, chunk=chunk, callback=callback)
            assert (got == want, err, state) == (True, 0, 4), (name, chunk)
            assert z.public.total == len(want)
            assert z.public.usedinput == len(c), name
            if name.startswith("gzip"):
                assert z.public.stype == E.ZSTRM_GZIP and z.public.crc == zlib.crc32(want)
            if name.startswith("zlib"):
                assert z.public.stype == E.ZSTRM_ZLIB and z.public.adler == zlib.adler32(want)


@pytest.mark.gpu
def test_zstrm_round_trip(engine):
    d = engine.corpus_mixed(20 << 20, seed=7).tobytes()
    for kind in ("gzip", "zlib", "raw"):
        c = engine.ZStrm(E.ZSTRM_DEFLATE | TYPES[kind], 6).compress(d)
        got, err, state = engine.ZStrm(E.ZSTRM_INFLATE, 0).decompress(c, chunk=(7 << 20) + 3)
        assert got == d and err == 0 and state == 4, kind


@pytest.mark.gpu
def test_zstrm_inflate_errors(engine):
    d = engine.corpus_text(200000, seed=4).tobytes()
    g = bytearray(gzip.compress(d))
    bad_crc = bytes(g[:-8]) + struct.pack("<I", zlib.crc32(d) ^ 1) + bytes(g[-4:])
    bad_len = bytes(g[:-4]) + struct.pack("<I", len(d) + 1)
    zl = zlib.compress(d)
    bad_adler = zl[:-1] + bytes([zl[-1] ^ 0x55])
    cases = [
        ("crc", E.ZSTRM_INFLATE, bad_crc, E.ZSTRM_ECHECKSUM),
        ("nocrc", E.ZSTRM_INFLATE | E.ZSTRM_NOCRC, bad_crc, 0),
        ("isize", E.ZSTRM_INFLATE, bad_len, E.ZSTRM_EBADDATA),
        ("adler", E.ZSTRM_INFLATE, bad_adler, E.ZSTRM_ECHECKSUM),
        ("noadler", E.ZSTRM_INFLATE | E.ZSTRM_NOADLER, bad_adler, 0),
        ("magic", E.ZSTRM_INFLATE, b"\x1f\x8c" + bytes(g[2:]), E.ZSTRM_EBADDATA),
        ("method", E.ZSTRM_INFLATE, b"\x1f\x8b\x07" + bytes(g[3:]), E.ZSTRM_EBADDATA),
        ("format", E.ZSTRM_INFLATE | E.ZSTRM_ZLIB, bytes(g), E.ZSTRM_EFORMAT),
        ("truncated", E.ZSTRM_INFLATE, bytes(g[:-3]), E.ZSTRM_ESRCEXHSTD),
        ("btype11", E.ZSTRM_INFLATE, b"\x07\x00", E.ZSTRM_EBADDATA),
        ("corrupt", E.ZSTRM_INFLATE, bytes(g[:10]) + b"\xff" * 64 + bytes(g[-8:]),
         E.ZSTRM_EDEFLATE),
    ]
    for name, flags, c, want in cases:
        z = engine.ZStrm(flags, 0)
        got, err, state = z.decompress(c, chunk=1 << 20)
        assert err == want and state == 4, (name, err)
    # zlib with a preset dictionary: the caller is told it is needed
    co = zlib.compressobj(6, zlib.DEFLATED, 15, zdict=b"dictionary words")
    zd = co.compress(d) + co.flush()
    z = engine.ZStrm(E.ZSTRM_INFLATE, 0)
    L = engine.load_library()
    buf = ctypes.create_string_buffer(zd, len(zd))
    L.zstrm_setsource(z._p, buf, len(zd))
    assert z.public.state == 2 and z.public.dictid == zlib.adler32(b"dictionary words")
    out = ctypes.create_string_buffer(16)
    assert L.zstrm_inflate(z._p, out, 16) == 0
    assert z.public.error == E.ZSTRM_EMISSINGDICT and z.public.state == 4


# ---- GPU: index-free parallel inflate of FLUSH-joined streams (row f4) -------

def _flushed(engine, stream, region=None, cap=None):
    L = engine.load_library()
    region = len(stream) if region is None else region
    cap = cap or max(4 * len(stream), 1 << 20)
    out = ctypes.create_string_buffer(cap)
    prod, used, err = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int32()
    c, a = ctypes.c_uint32(0xFFFFFFFF), ctypes.c_uint32(1)
    engine.prof_enable(True)
    r = L.jdgpu_inflate_flushed(stream, len(stream), region, out, cap, ctypes.byref(prod),
                                ctypes.byref(used), ctypes.byref(err), ctypes.byref(c),
                                ctypes.byref(a))
    kt = engine.prof_read()
    engine.prof_enable(False)
    assert r == 0
    parallel = "k_inflate_par" in kt or "k_inflate_lanes" in kt
    return out.raw[:prod.value], err.value, used.value, c.value ^ 0xFFFFFFFF, a.value, parallel


@pytest.mark.gpu
def test_inflate_flushed_paths(engine):
    d = engine.corpus_mixed(40 * BS + 123, seed=11).tobytes()
    # this library's block-mode stream: decoded in parallel
    s, _ = engine.deflate_blocks(d, level=6)
    got, err, used, crc, adler, par = _flushed(engine, s)
    assert (got == d, err, used, par) == (True, 0, len(s), True)
    assert crc == zlib.crc32(d) and adler == zlib.adler32(d)
    # zlib with a full flush every 64 KiB: independent blocks, a Huffman final block
    co = zlib.compressobj(6, zlib.DEFLATED, -15)
    z = b"".join(co.compress(d[o:o + BS]) + co.flush(zlib.Z_FULL_FLUSH) for o in range(0, len(d), BS))
    z += co.flush()
    got, err, used, crc, _, par = _flushed(engine, z)
    assert (got == d, err, used, par) == (True, 0, len(z), True)
    # sync flushes keep the window: the blocks are not independent -> serial
    co = zlib.compressobj(6, zlib.DEFLATED, -15)
    z = b"".join(co.compress(d[o:o + BS]) + co.flush(zlib.Z_SYNC_FLUSH) for o in range(0, len(d), BS))
    z += co.flush()
    got, err, used, crc, _, par = _flushed(engine, z)
    assert (got == d, err, used, crc) == (True, 0, len(z), zlib.crc32(d))
    # a plain zlib stream (no markers) -> serial
    z = _raw(d, 9)
    got, err, used, crc, _, par = _flushed(engine, z)
    assert (got == d, err, par) == (True, 0, False)
    # stored blocks whose payload holds the marker bytes: false markers -> serial
    dm = (b"ab\x00\x00\xff\xffcd" * 20000)[:3 * BS + 7]
    s, _ = engine.deflate_blocks(dm, level=0)
    got, err, used, _, _, par = _flushed(engine, s)
    assert (got == dm, err, used) == (True, 0, len(s))
    # a container trailer after the stream (region excludes it)
    s, _ = engine.deflate_blocks(d, level=1)
    got, err, used, _, _, par = _flushed(engine, s + b"TRAILER!", region=len(s))
    assert (got == d, err, used, par) == (True, 0, len(s), True)
    # too small a buffer reports the overflow (the caller grows it)
    _, err, _, _, _, _ = _flushed(engine, engine.deflate_blocks(d, level=6)[0], cap=BS)
    assert err == 9


@pytest.mark.gpu
def test_zstrm_inflate_own_gzip_is_parallel(engine):
    d = engine.corpus_text(9 << 20, seed=8).tobytes()
    c = engine.ZStrm(E.ZSTRM_DEFLATE | E.ZSTRM_GZIP, 6).compress(d)
    engine.prof_enable(True)
    got, err, state = engine.ZStrm(E.ZSTRM_INFLATE, 0).decompress(c, chunk=1 << 22)
    kt = engine.prof_read()
    engine.prof_enable(False)
    assert (got == d, err, state) == (True, 0, 4)
    assert "k_inflate_par" in kt or "k_inflate_lanes" in kt


@pytest.mark.gpu
def test_zstrm_preset_dictionary(engine):
    """zstrm_setdctnr (zstrm.c:327-390): a zlib stream with FDICT inflates
    with its dictionary (the wrong one is EBADDICT); a deflate with one
    writes FDICT/DICTID that zlib accepts with that dictionary."""
    E = engine.engine
    L = engine.load_library()
    d = engine.corpus_text(200000, seed=51).tobytes()
    dic = d[:40000]
    data = d[40000:]
    co = zlib.compressobj(6, zlib.DEFLATED, 15, zdict=dic)
    zd = co.compress(data) + co.flush()
    for use, want in ((dic, E.ZSTRM_OK), (b"other dictionary", E.ZSTRM_EBADDICT)):
        z = engine.ZStrm(E.ZSTRM_INFLATE | E.ZSTRM_ZLIB, 0)
        buf = ctypes.create_string_buffer(zd, len(zd))
        L.zstrm_setsource(z._p, buf, len(zd))
        assert z.public.state == 2
        L.zstrm_setdctnr(z._p, use, len(use))
        if want == E.ZSTRM_OK:
            out = ctypes.create_string_buffer(len(data) + 100)
            n = L.zstrm_inflate(z._p, out, len(data) + 100)
            assert n == len(data) and out.raw[:n] == data
            assert z.public.error == 0 and z.public.state == 4
        else:
            assert z.public.error == want and z.public.state == 4
        z.close()
    # a raw stream is past its (empty) header once the source is set
    # (state 3), so a dictionary then is misuse, as in the reference
    co = zlib.compressobj(6, zlib.DEFLATED, -15, zdict=dic)
    raw = co.compress(data) + co.flush()
    z = engine.ZStrm(E.ZSTRM_INFLATE | E.ZSTRM_DFLT, 0)
    buf = ctypes.create_string_buffer(raw, len(raw))
    L.zstrm_setsource(z._p, buf, len(raw))
    assert z.public.state == 3
    L.zstrm_setdctnr(z._p, dic, len(dic))
    assert z.public.error == E.ZSTRM_EINCORRECTUSE and z.public.state == 4
    z.close()
    # deflate with a dictionary (set once the target is, state 1): FDICT +
    # DICTID, readable by zlib with it
    z = engine.ZStrm(E.ZSTRM_DEFLATE | E.ZSTRM_ZLIB, 6)
    out = []

    def ofn(buf, size, user):
        out.append(ctypes.string_at(buf, size))
        return size
    cb = E.ZSTRM_OFN(ofn)
    L.zstrm_settargetfn(z._p, cb, None)
    L.zstrm_setdctnr(z._p, dic, len(dic))
    assert z.public.error == 0 and z.public.dict == 1
    assert L.zstrm_deflate(z._p, data, len(data)) == len(data)
    L.zstrm_flush(z._p, 1)
    z.close()
    c = b"".join(out)
    assert c[1] & 0x20 and int.from_bytes(c[2:6], "big") == zlib.adler32(dic)
    assert zlib.decompressobj(15, zdict=dic).decompress(c) == data


@pytest.mark.gpu
def test_gzip_inflate_on_threads(engine):
    """zstrm gzip/zlib decodes on 8 threads at once, 32 KiB source reads:
    every call carries the CRC-32 / Adler-32 update, which each instance
    computes in its own scratch (no engine lock), so the instances overlap;
    every container must decode exactly, trailers checked"""
    import gzip as _gz
    import threading
    datas = [engine.corpus_text(600_000, seed=300 + k).tobytes() for k in range(8)]
    conts = [_gz.compress(d, 6) if k % 2 == 0 else zlib.compress(d, 6) for k, d in enumerate(datas)]
    res = [None] * 8

    def work(k):
        fmt = E.ZSTRM_GZIP if k % 2 == 0 else E.ZSTRM_ZLIB
        z = E.ZStrm(E.ZSTRM_INFLATE | fmt)
        res[k] = z.decompress(conts[k], chunk=65536, callback=True, readsize=32768)
        z.close()

    ths = [threading.Thread(target=work, args=(k,)) for k in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for k in range(8):
        out, err, state = res[k]
        assert err == 0 and out == datas[k], (k, err, state)

"""Streaming contract of the drop-in inflator (inflator.c:765-903 of the
reference): input fed in chunks with final=0 throughout, as the reference's
own zstrm.c:926 does in callback mode.  Every call must deliver exactly what
the reference delivers for the input given so far (the oracle's decode of
that prefix, oracle/jdoracle.py inflate_call), the call in which the final
block ends must return INFLT_OK, and `source` must stop on the first byte
after the stream.  GPU tests, through the C ABI."""
import ctypes
import os
import subprocess
import zlib

import pytest

from jdeflate_amd import engine as E

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRAILER = bytes(range(0xA0, 0xA8))        # 8 bytes after the stream (a gzip trailer's size)


def zraw(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, zdict=None):
    kw = {"zdict": zdict} if zdict else {}
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy, **kw)
    return c.compress(data) + c.flush()


def streams(engine):
    J = engine
    text = J.corpus_text(200_000, seed=11).tobytes()
    mixed = J.corpus_mixed(150_000, seed=12).tobytes()
    blk, _ = J.deflate_blocks(text, level=6)
    return {
        "blocks_L6": (blk, text),
        "zlib_L6": (zraw(text), text),
        "zlib_L1_mixed": (zraw(mixed, 1), mixed),
        "zlib_L9_huffonly": (zraw(text[:50_000], 9, zlib.Z_HUFFMAN_ONLY), text[:50_000]),
        "zlib_stored": (zraw(mixed[:70_000], 0), mixed[:70_000]),
        "zlib_fixed": (zraw(text[:30_000], 6, zlib.Z_FIXED), text[:30_000]),
        "tiny": (zraw(b"abc"), b"abc"),
        "empty": (zraw(b""), b""),
    }


def check_trace(oracle, comp, trace, chunk, final_mode, delivered):
    """every call's delivered bytes equal the reference's for that prefix:
    its result code, and the bytes themselves -- everything the calls so
    far delivered (delivered[:got], the calls' outputs in order) against the
    oracle's decode of the input given so far"""
    for k, r, got, _ in trace:
        if r == E.INFLT_TGTEXHSTD:
            continue
        n = min(len(comp), (k + 1) * chunk)
        fin = final_mode == "last" and n >= len(comp)
        rr, err, out, _ = oracle.inflate_call(comp, n, 1 << 24, fin)
        assert r == rr, (k, r, rr, err)
        assert got == len(out), (k, got, len(out))
        assert delivered[:got] == out, (k, got)


@pytest.mark.parametrize("chunk", [7, 333, 4096, 65536, 1 << 30])
def test_final0_chunks(engine, oracle, chunk):
    for name, (comp, data) in streams(engine).items():
        if chunk == 7 and len(comp) > 5000:
            continue
        src = comp + TRAILER
        inf = E.Inflator()
        trace = []
        out, r, err = inf.decompress(src, chunk=chunk, tgt=1 << 20, final="never", trace=trace)
        assert r == E.INFLT_OK, (name, r, err)
        assert out == data, name
        _, _, _, cons = oracle.inflate(comp, len(data) + 64)
        assert cons == len(comp)
        assert inf.consumed == len(comp), (name, inf.consumed, len(comp))
        check_trace(oracle, src, trace, chunk, "never", out)


@pytest.mark.parametrize("tgt", [1, 1000, 32768])
def test_small_targets_final0(engine, oracle, tgt):
    comp, data = streams(engine)["zlib_L6"]
    inf = E.Inflator()
    out, r, err = inf.decompress(comp + TRAILER, chunk=20_000, tgt=tgt, final="never")
    assert (r, out) == (E.INFLT_OK, data)
    assert inf.consumed == len(comp)


@pytest.mark.parametrize("tgt", [1000, 65536])
def test_small_targets_decode_ahead(engine, tgt):
    """This library's FLUSH-joined blocks in 300 KB pieces through small
    targets: the segments are decoded in parallel ahead of the target and
    drained over the following calls (TGTEXHSTD with nothing consumed)."""
    data = engine.corpus_text(2_000_000, seed=13).tobytes()
    comp, _ = engine.deflate_blocks(data, level=6)
    inf = E.Inflator()
    trace = []
    out, r, err = inf.decompress(comp + TRAILER, chunk=300_000, tgt=tgt, final="never",
                                 trace=trace)
    assert (r, out) == (E.INFLT_OK, data)
    assert inf.consumed == len(comp)


def test_truncated_final1_is_inputend(engine, oracle):
    for name, (comp, data) in streams(engine).items():
        if len(comp) < 40:
            continue
        cut = comp[:len(comp) - 17]
        out, r, err = E.Inflator().decompress(cut, chunk=5000)
        rr, rerr, rout, _ = oracle.inflate_call(cut, len(cut), 1 << 24, True)
        assert (r, err) == (E.INFLT_ERROR, E.INFLT_EINPUTEND) == (rr, rerr), name
        assert out == rout, name


def test_truncated_final0_then_misuse(engine):
    comp, data = streams(engine)["zlib_L6"]
    inf = E.Inflator()
    out, r, err = inf.decompress(comp[:-30], chunk=10_000, final="never")
    # input exhausted without final: SRCEXHSTD, then the empty call is misuse
    # (validate :744-750)
    assert (r, err) == (E.INFLT_ERROR, E.INFLT_EINCORRECTUSE)
    assert data.startswith(out) and len(out) > len(data) // 2


def test_corrupt_midstream(engine, oracle):
    comp, data = streams(engine)["zlib_L6"]
    bad = bytearray(comp)
    for i in range(5000, 5040):
        bad[i] = 0xFF
    out, r, err = E.Inflator().decompress(bytes(bad), chunk=3000, final="never")
    rr, rerr, rout, _ = oracle.inflate_call(bytes(bad), len(bad), 1 << 24, False)
    assert (r, err) == (rr, rerr)
    assert out == rout


def test_dictionary_final0(engine):
    J = engine
    d = J.corpus_text(40_000, seed=5).tobytes()
    data = J.corpus_text(90_000, seed=6).tobytes()
    comp = zraw(data, 6, zdict=d[-32768:])
    inf = E.Inflator()
    inf.setdctnr(d)
    out, r, err = inf.decompress(comp + TRAILER, chunk=3000, final="never")
    assert (r, out) == (E.INFLT_OK, data)
    assert inf.consumed == len(comp)


def test_large_flush_joined_final0(engine):
    """3 MiB of this library's block-mode output in 1 MiB chunks: the parallel
    prefix path resumes at a verified marker each time"""
    J = engine
    data = J.corpus_text(3 << 20, seed=21).tobytes()
    comp, _ = J.deflate_blocks(data, level=6)
    inf = E.Inflator()
    out, r, err = inf.decompress(comp + TRAILER, chunk=1 << 20, tgt=1 << 22, final="never")
    assert (r, out) == (E.INFLT_OK, data)
    assert inf.consumed == len(comp)


def test_resume_api_parallel_prefix(engine):
    """jdgpu_inflate_resume on a whole FLUSH-joined stream decodes its
    segments in parallel and reports the exact end"""
    import ctypes
    J = engine
    L = J.load_library()
    data = J.corpus_text(2 << 20, seed=22).tobytes()
    comp, sizes = J.deflate_blocks(data, level=6)
    out = ctypes.create_string_buffer(len(data) + 65536)
    res = E.InflateResult()
    r = L.jdgpu_inflate_resume(b"\0", 0, comp + TRAILER, len(comp) + 8, len(comp) + 8, 0, out,
                               len(data) + 65536, ctypes.byref(res), 0, None, None)
    assert r == 0 and res.error == 0
    assert res.produced == len(data) and out.raw[:len(data)] == data
    assert res.consumed == len(comp)
    assert res.parallel == len(sizes)
    assert (res.resumebit, res.resumeout) == (len(comp) * 8, len(data))


def test_resume_api_input_end_has_no_resume_point(engine):
    """a one-shot decode whose input runs out reports
    INFLT_EINPUTEND and no resume point (the decoder state is not kept);
    decoding the whole stream again from its start gives the data, and the
    resumable decoder (jdgpu_istream) continues the same cut input exactly."""
    import ctypes
    J = engine
    L = J.load_library()
    data = J.corpus_text(600_000, seed=23).tobytes()
    comp = zraw(data)
    cut = len(comp) // 2
    out = ctypes.create_string_buffer(len(data) + 65536)
    res = E.InflateResult()
    r = L.jdgpu_inflate_resume(b"\0", 0, comp[:cut], cut, cut, 0, out, len(data) + 65536,
                               ctypes.byref(res), 0, None, None)
    assert r == 0 and res.error == E.INFLT_EINPUTEND
    assert (res.resumebit, res.resumeout) == (0, 0)
    assert 0 < res.produced < len(data) and out.raw[:res.produced] == data[:res.produced]
    s = E.IStream()
    got = bytearray()
    st, err, prod, cons, _ = s.inflate(comp[:cut], len(data))
    got += s.out.raw[:prod]
    assert (st, cons, prod) == (E.IS_NEEDINPUT, cut, res.produced)
    st, err, prod, cons, _ = s.inflate(comp[cut:], len(data))
    got += s.out.raw[:prod]
    assert (st, err) == (E.IS_ENDED, 0) and bytes(got) == data


C_CALLER = r'''
/* a caller written like zstrm.c:900-930 in callback mode: input in small
 * reads, final = 0 on every call, a 32 KiB target drained between calls */
#include <jdeflate/inflator.h>
#include <stdio.h>
#include <stdlib.h>
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb");
    FILE* g = fopen(argv[2], "wb");
    static uint8 in[4096], out[32768];
    size_t fed = 0, n;
    eINFLTResult r = INFLT_SRCEXHSTD;
    TInflator* z = inflator_create(0, NULL);
    if (!f || !g || !z) return 2;
    while (r == INFLT_SRCEXHSTD && (n = fread(in, 1, sizeof in, f)) > 0) {
        inflator_setsrc(z, in, n);
        do {
            inflator_settgt(z, out, sizeof out);
            r = inflator_inflate(z, 0);
            fwrite(out, 1, inflator_tgtend(z), g);
        } while (r == INFLT_TGTEXHSTD);
        fed += (r == INFLT_OK) ? inflator_srcend(z) : n;
    }
    printf("%d %u %zu\n", (int) r, (unsigned) z->error, fed);
    inflator_destroy(z);
    fclose(g);
    return r == INFLT_OK ? 0 : 1;
}
'''


def test_c99_callback_caller(engine, built_lib, tmp_path):
    J = engine
    data = J.corpus_text(300_000, seed=31).tobytes()
    comp = zraw(data, 9)
    (tmp_path / "in.bin").write_bytes(comp + TRAILER)
    (tmp_path / "caller.c").write_text(C_CALLER)
    exe = tmp_path / "caller"
    inc = os.path.join(ROOT, "include")
    libdir = os.path.dirname(built_lib)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", inc, str(tmp_path / "caller.c"),
                    "-o", str(exe), "-L", libdir, "-ljdeflate_amd", "-Wl,-rpath," + libdir],
                   check=True)
    p = subprocess.run([str(exe), str(tmp_path / "in.bin"), str(tmp_path / "out.bin")],
                       capture_output=True, text=True, timeout=120)
    r, err, fed = p.stdout.split()
    assert (int(r), int(err), int(fed)) == (E.INFLT_OK, 0, len(comp))
    assert (tmp_path / "out.bin").read_bytes() == data


def test_istream_decodes_each_bit_once(engine, oracle):
    """The resumable decoder behind the drop-in inflator: 4 KiB input pieces,
    32 KiB targets, a foreign (zlib) stream.  Between calls only the bytes of
    an incomplete token or block header stay with the host (jdgpu_istream
    carried bytes), never a whole block as a resume-at-block-start design
    would keep, and the output equals the oracle's."""
    data = engine.corpus_text(400_000, seed=41).tobytes()
    comp = zraw(data, 6)
    s = E.IStream()
    out = bytearray()
    pos = 0
    calls = 0
    while True:
        piece = comp[pos:pos + 4096]
        st, err, prod, cons, _ = s.inflate(piece, 32768)
        out += s.out.raw[:prod]
        calls += 1
        if st == E.IS_FULL:
            pos += cons
            continue
        pos += cons
        if st != E.IS_NEEDINPUT:
            break
    assert (st, err) == (E.IS_ENDED, 0)
    assert bytes(out) == data
    assert pos == len(comp)
    launches, par, carried = s.stats()
    ncalls = -(-len(comp) // 4096)
    assert carried <= 600 * ncalls, (carried, ncalls)
    assert launches <= calls


def test_istream_pending_copy_tiny_targets(engine):
    """Back-references split by 1-byte and 7-byte targets (copybytes
    :1214-1290): the pending copy resumes in the next call, with or without
    new input."""
    data = (b"abcabcabcabc" * 500 + bytes(3000) + b"xyz" * 900) * 3
    for tgt in (1, 7, 1000):
        comp = zraw(data, 9)
        s = E.IStream()
        out = bytearray()
        pos = 0
        while True:
            st, err, prod, cons, _ = s.inflate(comp[pos:], tgt)
            out += s.out.raw[:prod]
            pos += cons
            if st != E.IS_FULL:
                break
        assert (st, err) == (E.IS_ENDED, 0), tgt
        assert bytes(out) == data, tgt
        assert pos == len(comp)


def test_dropin_inflate_output_over_4gib(engine):
    """One inflator_inflate call whose output is 4.25 GiB (68 x 64 MiB of
    FLUSH-joined text blocks, then the END terminator): no 4 GiB limit in the
    drop-in path; every 64 MiB piece of the output is checked."""
    import ctypes
    import numpy as np
    J = engine
    L = J.load_library()
    piece = J.corpus_text(64 << 20, seed=51)
    cap = J.bound(piece.size)
    cbuf = np.empty(cap, dtype=np.uint8)
    csz = np.empty(1024, dtype=np.uint32)
    n = L.jdgpu_deflate(piece.ctypes.data_as(ctypes.c_char_p), piece.size, 65536, 6, 0, 2,
                        cbuf.ctypes.data, cap, csz.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    assert n > 0
    reps = 68
    comp = np.concatenate([np.tile(cbuf[:n], reps), np.frombuffer(b"\x01\x00\x00\xff\xff", np.uint8)])
    total = reps * piece.size
    assert total > (4 << 30)
    out = np.zeros(total + 16, dtype=np.uint8)
    inf = E.Inflator()
    s = inf.public
    s.source = s.sbgn = comp.ctypes.data
    s.send = comp.ctypes.data + comp.size
    s.target = s.tbgn = out.ctypes.data
    s.tend = out.ctypes.data + out.size
    r = inf.inflate(1)
    assert r == E.INFLT_OK, (r, s.error)
    assert inf.tgtend() == total
    assert inf.srcend() == comp.size
    for i in range(reps):
        assert np.array_equal(out[i * piece.size:(i + 1) * piece.size], piece), i


def test_many_instances_on_threads(engine):
    """20 drop-in inflators alive at once, one per thread, 32 KiB reads with
    final=0: the first 16 run on hardware queues of their own, the rest on
    the shared ones (jd_engine.cpp is_stream_create); every instance must
    decode its own stream exactly, whichever queue it got"""
    import threading
    datas = [engine.corpus_text(400_000, seed=100 + k).tobytes() for k in range(20)]
    comps = [engine.deflate_blocks(d, level=6)[0] if k % 2 else zraw(d) for k, d in enumerate(datas)]
    infs = [E.Inflator() for _ in range(20)]
    res = [None] * 20

    def work(k):
        res[k] = infs[k].decompress(comps[k] + TRAILER, chunk=32768, tgt=65536, final="never")

    ths = [threading.Thread(target=work, args=(k,)) for k in range(20)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for k in range(20):
        out, r, err = res[k]
        assert (r, out == datas[k]) == (E.INFLT_OK, True), (k, r, err)
        assert infs[k].consumed == len(comps[k]), k


def test_shared_queue_instances_are_reported(engine):
    """jdgpu_istream_queue: at most 16 live instances hold a hardware queue
    of their own; the ones past that share the process's queues and say so"""
    import gc
    gc.collect()
    ins = [E.IStream() for _ in range(20)]
    own = [s.own_queue() for s in ins]
    assert sum(own) <= 16 and own.count(False) >= 4, own
    for s in ins:
        s.close()
    s2 = E.IStream()
    assert s2.own_queue()              # the freed queues are handed out again
    s2.close()


@pytest.mark.parametrize("rewrite", [False, True])
def test_cached_input_rewritten_in_place(engine, rewrite):
    """After a full target the rest of the caller's buffer stays staged on
    the device; a caller that rewrites the middle of that rest in place (same
    address, same first and last bytes) must get the new bytes decoded, as
    the reference reads its source on every call"""
    data = engine.corpus_text(900_000, seed=71).tobytes()
    comp = zraw(data)
    buf = ctypes.create_string_buffer(comp, len(comp))
    base = ctypes.addressof(buf)
    s = E.IStream()
    out, off, first = b"", 0, True
    while True:
        st, err, prod, cons, _ = s.inflate(len(comp) - off, 65536, src_addr=base + off)
        out += s.out.raw[:prod]
        off += cons
        if first and rewrite:
            mid = off + (len(comp) - off) // 2
            ctypes.memmove(base + mid, b"\xa5" * 4096, 4096)
        first = False
        if st != E.IS_FULL:
            break
    s.close()
    if rewrite:
        assert st == E.IS_ERROR or out != data     # the rewritten bytes were read
    else:
        assert out == data and st == E.IS_ENDED


def _calls_per_second(comp, ncalls, rewrite_at=None):
    """ncalls calls of 64 KiB targets over one caller buffer holding all of
    comp (zlib, so no sync markers; chunk-parallel rounds off): each call
    passes the whole rest of the buffer.  -> (seconds per call, output,
    final status)"""
    import time
    buf = ctypes.create_string_buffer(comp, len(comp))
    base = ctypes.addressof(buf)
    s = E.IStream()
    s.fsp(0)
    out, off, k = bytearray(), 0, 0
    t0 = time.perf_counter()
    st = E.IS_FULL
    while st == E.IS_FULL and k < ncalls:
        st, err, prod, cons, _ = s.inflate(len(comp) - off, 65536, src_addr=base + off)
        out += s.out.raw[:prod]
        off += cons
        k += 1
        if k == 1 and rewrite_at is not None:
            ctypes.memmove(base + off + rewrite_at, b"\xa5" * 4096, 4096)
    dt = (time.perf_counter() - t0) / k
    s.close()
    return dt, bytes(out), st


def test_cached_window_is_bounded(engine):
    """after a full target only a bounded window of the rest of
    the caller's buffer is kept staged and re-verified (1 MiB here, 4x what
    a call consumed), so a call's host work does not grow with the size of
    the rest: 150 calls over a 48 MB source cost about what they cost over
    a 3 MB one (re-hashing the whole rest made it ~5x)."""
    data = engine.corpus_text(120_000_000, seed=72, threads=16).tobytes()
    comp = zlib.compress(data, 1)[2:-4]
    big = comp[:48_000_000]
    small = comp[:3_000_000]
    _calls_per_second(small, 20)                     # warm up
    t_small, o_small, s_small = _calls_per_second(small, 60)
    t_big, o_big, s_big = _calls_per_second(big, 60)
    assert s_small == s_big == E.IS_FULL             # 60 full 64 KiB targets each
    assert o_small == o_big == data[:len(o_big)]
    assert t_big < 2.0 * t_small, (t_big, t_small)


def test_cached_rewrite_past_the_window(engine):
    """a rewrite of the caller's buffer beyond the verified window (5 MB
    ahead of the call's position) is read too: bytes past the window are
    staged from the host when the decoder gets there"""
    data = engine.corpus_text(30_000_000, seed=73, threads=16).tobytes()
    comp = zlib.compress(data, 1)[2:-4]
    _, out, st = _calls_per_second(comp, 10 ** 6, rewrite_at=5_000_000)
    assert st == E.IS_ERROR or out != data
    _, out, st = _calls_per_second(comp, 10 ** 6)
    assert st == E.IS_ENDED and out == data

"""The parallel resume (k_inflate_rpar) behind the
drop-in inflator: the span at hand decoded by 256 self-synchronising
segment walks (four waves) instead of the
one-wave serial decoder.  Every call's result must be the
serial decoder's, bit for bit -- status, error code, bytes produced and
consumed, and the bytes themselves -- on this library's streams, zlib's
(levels 1/6/9, Huffman-only, fixed codes, stored), with a dictionary, on
truncated and corrupted input, through input pieces and targets of many
sizes.  The serial decoder is itself checked call by call against the
oracle's per-prefix decode (tests/test_inflator_stream.py), and
test_rpar_calls_equal_oracle checks the parallel resume's calls against the
oracle directly."""
import zlib

import pytest

from jdeflate_amd import engine as E

pytestmark = pytest.mark.gpu


def zraw(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, zdict=None):
    kw = {"zdict": zdict} if zdict else {}
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy, **kw)
    return c.compress(data) + c.flush()


def run(comp, piece, tgt, rpar, dict_=None, limit=100000):
    """feed `comp` in pieces of `piece` bytes; -> list of call results + output"""
    s = E.IStream(dict_)
    s.rpar(1 if rpar else 0)
    out = bytearray()
    trace = []
    pos = 0
    for _ in range(limit):
        p = comp[pos:pos + piece]
        st, err, prod, cons, _ = s.inflate(p, tgt)
        out += s.out.raw[:prod]
        trace.append((st, err, prod, cons))
        pos += cons
        if st == E.IS_FULL:
            continue
        if st != E.IS_NEEDINPUT or pos >= len(comp):
            break
    launches = s.rpar()
    s.close()
    return trace, bytes(out), launches


def corpora(J):
    text = J.corpus_text(600_000, seed=31).tobytes()
    mixed = J.corpus_mixed(400_000, seed=32).tobytes()
    blk, _ = J.deflate_blocks(text, level=6)
    blk9, _ = J.deflate_blocks(mixed, level=9)
    return {
        "blocks_L6_text": blk,
        "blocks_L9_mixed": blk9,
        "zlib_L6_text": zraw(text),
        "zlib_L1_text": zraw(text, 1),
        "zlib_L9_mixed": zraw(mixed, 9),
        "zlib_huffonly": zraw(text[:200_000], 9, zlib.Z_HUFFMAN_ONLY),
        "zlib_fixed": zraw(text[:100_000], 6, zlib.Z_FIXED),
        "zlib_stored": zraw(mixed[:150_000], 0),
        "runs": zraw(bytes(50_000) + b"ab" * 40_000 + bytes(30_000), 9),
    }


@pytest.mark.parametrize("piece,tgt", [(32768, 65536), (4096, 1 << 20), (100_000, 7000),
                                       (1 << 20, 65536), (777, 300)])
def test_rpar_equals_serial(engine, piece, tgt):
    for name, comp in corpora(engine).items():
        a, oa, la = run(comp, piece, tgt, True)
        b, ob, lb = run(comp, piece, tgt, False)
        assert lb == 0
        assert oa == ob, (name, len(oa), len(ob))
        assert a == b, (name, next((i, x, y) for i, (x, y) in enumerate(zip(a, b)) if x != y))
        assert a[-1][0] == E.IS_ENDED, name


@pytest.mark.parametrize("piece", [32768, 5000])
def test_rpar_calls_equal_oracle(engine, oracle, piece):
    """Every call of the parallel resume against the oracle itself, not the
    serial decoder: with a target no call fills, the bytes delivered after
    the input given so far (all calls' outputs in order) are the oracle's
    decode of that prefix, and the status is the oracle's (NEEDINPUT while
    the input runs out, ENDED with the stream's exact end)."""
    J = engine
    text = J.corpus_text(300_000, seed=37).tobytes()
    mixed = J.corpus_mixed(200_000, seed=38).tobytes()
    cases = [J.deflate_blocks(text, level=6)[0], zraw(text), zraw(mixed, 9),
             zraw(text[:120_000], 6, zlib.Z_FIXED)]
    for comp in cases:
        trace, out, launches = run(comp, piece, 1 << 22, True)
        assert launches > 0
        fed = got = 0
        for st, err, prod, cons in trace:
            fed += cons
            got += prod
            rr, rerr, rout, rcons = oracle.inflate_call(comp, fed, 1 << 24, False)
            assert out[:got] == rout, (len(comp), fed, got, len(rout))
            if st == E.IS_ENDED:
                assert (rr, rcons) == (0, fed)
            else:
                assert st == E.IS_NEEDINPUT and rr == 1, (st, rr, rerr)


def test_rpar_is_used_on_text(engine):
    """32 KiB pieces of text streams go through the parallel decoder"""
    J = engine
    text = J.corpus_text(2 << 20, seed=33).tobytes()
    for comp in (J.deflate_blocks(text, level=6)[0], zraw(text)):
        tr, out, launches = run(comp, 32768, 65536, True)
        assert out == text and tr[-1][0] == E.IS_ENDED
        assert launches >= len(comp) // 32768 // 2, launches


def test_rpar_dictionary(engine):
    J = engine
    d = J.corpus_text(40_000, seed=34).tobytes()
    data = J.corpus_text(300_000, seed=35).tobytes()
    comp = zraw(data, 6, zdict=d[-32768:])
    a, oa, la = run(comp, 32768, 65536, True, dict_=d)
    b, ob, _ = run(comp, 32768, 65536, False, dict_=d)
    assert oa == ob == data and a == b and la > 0


def test_rpar_truncated_and_corrupt(engine):
    J = engine
    text = J.corpus_text(300_000, seed=36).tobytes()
    comp = zraw(text)
    cases = [comp[:len(comp) // 2], comp[:-3]]
    for at in (20_000, 50_001, 90_000):
        bad = bytearray(comp)
        for i in range(at, at + 40):
            bad[i] ^= 0x5A
        cases.append(bytes(bad))
    for c in cases:
        for piece in (32768, 5000):
            a, oa, _ = run(c, piece, 65536, True)
            b, ob, _ = run(c, piece, 65536, False)
            assert oa == ob and a == b


def test_instances_on_threads(engine):
    """Independent decoder instances on 8 threads at once (the reference's
    threading model, inflator.h): each has its own HIP stream and state; the
    engine lock is held only around shared workspace.  Every instance's
    output is exact, for this library's streams and zlib's, while the others
    run (and the marker-parallel path, which takes the shared workspace,
    runs in some of them)."""
    import threading
    J = engine
    jobs = []
    for k in range(8):
        data = J.corpus_text(400_000 + 50_000 * k, seed=100 + k).tobytes()
        comp = J.deflate_blocks(data, level=6)[0] if k % 2 else zraw(data, 1 + k % 9)
        piece = 32768 if k < 6 else 300_000
        jobs.append((comp, data, piece))
    res = [None] * len(jobs)

    def work(i):
        comp, data, piece = jobs[i]
        res[i] = run(comp, piece, 65536, True)

    ths = [threading.Thread(target=work, args=(i,)) for i in range(len(jobs))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for (comp, data, piece), r in zip(jobs, res):
        trace, out, launches = r
        assert out == data and trace[-1][0] == E.IS_ENDED

"""Single-window stream deflate on the GPU against the
oracle's single-stream restatement (jdo_deflate: the reference fed the whole
input with one deflator_setsrc, then DEFLT_END or DEFLT_FLUSH).  Bit-exact.

The sizes cover no slide (n <= 128 KiB), one and several window slides
(deflator.c:1818-1862), and stream ends right around a slide, where the
last positions' matches read the bytes the slid window holds past the end.
"""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

C1 = b"The quick brown fox jumps over the lazy dog. "


def inputs(J):
    rng = np.random.default_rng(5)
    text = J.corpus_text(3 << 20, seed=31).tobytes()
    mixed = J.corpus_mixed(2 << 20, seed=32).tobytes()
    return {
        "empty": b"",
        "one": b"x",
        "three": b"abc",
        "short": text[:100],
        "64k": text[:65536],
        "64k+1": text[:65537],
        "128k": text[:131072],
        "200k": text[:200000],
        "text1m": text[:1 << 20],
        "text3m": text,
        "mixed2m": mixed,
        "random": rng.integers(0, 256, 300000, dtype=np.uint8).tobytes(),
        "zeros": bytes(300000),
        "c1": (C1 * (2 ** 20 // len(C1) + 1))[:2 ** 20],
    }


def check(J, O, data, level, flush=1):
    g = J.deflate_stream(data, level=level, flush=flush)
    r = O.deflate(data, level=level, flush=flush)
    assert len(g) == len(r) and g == r, (len(data), level, flush, len(g), len(r))
    return g


def test_known_answer_c1(engine, oracle):
    """configs[0]: 1 MiB of repeated ASCII, level 6, one stream -> 3,117 B
    (the reference's own output)."""
    data = (C1 * (2 ** 20 // len(C1) + 1))[:2 ** 20]
    g = check(engine, oracle, data, 6)
    assert len(g) == 3117
    assert zlib.decompressobj(-15).decompress(g) == data


@pytest.mark.parametrize("level", [1, 2, 3, 4, 5, 6, 7, 8, 9])
def test_stream_parity(engine, oracle, level):
    for name, data in inputs(engine).items():
        g = check(engine, oracle, data, level)
        assert zlib.decompressobj(-15).decompress(g) == data, name


@pytest.mark.parametrize("level", [6, 9])
def test_stream_flush_terminator(engine, oracle, level):
    data = engine.corpus_text(300000, seed=9).tobytes()
    g = check(engine, oracle, data, level, flush=2)
    assert g[-4:] == b"\x00\x00\xff\xff"


def test_stream_ends_around_slides(engine, oracle):
    """Stream ends just before, at and after the first and second window
    slides: the tail records over the slid window's bytes."""
    text = engine.corpus_text(400000, seed=77).tobytes()
    mixed = engine.corpus_mixed(400000, seed=78).tobytes()
    for level, bases in ((6, (131072, 131072 + 98304)), (3, (65536, 65536 + 32768))):
        for base in bases:
            for k in range(-300, 700, 41):
                for data in (text, mixed):
                    check(engine, oracle, data[:base + k], level)


def test_stream_level0(engine, oracle):
    for n in (0, 1, 65535, 65536, 200000):
        data = bytes(range(256)) * (n // 256 + 1)
        check(engine, oracle, data[:n], 0)
        check(engine, oracle, data[:n], 0, flush=2)


def test_dropin_single_window(engine, oracle):
    """deflator_* with DEFLT_SINGLEWINDOW: the reference's own output for any
    feeding pattern (the reference is chunking-invariant)."""
    J = engine
    data = J.corpus_text(400000, seed=14).tobytes()
    for level in (1, 6, 9):
        want = oracle.deflate(data, level=level)
        for chunk, tgt in ((1 << 30, 1 << 20), (7919, 1000), (65536, 13)):
            d = J.Deflator(level, flags=J.engine.DEFLT_SINGLEWINDOW)
            assert d.compress(data, chunk=chunk, tgt=tgt) == want, (level, chunk, tgt)
            d.close()
    # configs[0] through the drop-in API
    c1 = (C1 * (2 ** 20 // len(C1) + 1))[:2 ** 20]
    d = J.Deflator(6, flags=J.engine.DEFLT_SINGLEWINDOW)
    out = d.compress(c1, chunk=65536, tgt=4096)
    d.close()
    assert len(out) == 3117 and out == oracle.deflate(c1, level=6)


@pytest.mark.parametrize("level", [0, 1, 4, 6, 9])
def test_stream_dictionary(engine, oracle, level):
    """deflator_setdctnr (deflator.c:2106-2167): the dictionary primes the
    window; checked against the oracle and against zlib's zdict inflate."""
    text = engine.corpus_text(300000, seed=41).tobytes()
    for dsize in (1, 3, 4, 5, 1000, 32768, 40000):
        dic, data = text[:dsize], text[dsize:dsize + 150000]
        g = engine.deflate_stream(data, level=level, dictionary=dic)
        r = oracle.deflate_dict(dic, data, level=level)
        assert g == r, (level, dsize)
        assert zlib.decompressobj(-15, zdict=dic[-32768:]).decompress(g) == data
    # an empty input after a dictionary: only the terminator
    assert engine.deflate_stream(b"", level=level, dictionary=text[:100]) == \
        oracle.deflate_dict(text[:100], b"", level=level)


def test_dropin_setdctnr(engine, oracle):
    J = engine
    text = J.corpus_text(200000, seed=42).tobytes()
    d = J.Deflator(6, flags=J.engine.DEFLT_SINGLEWINDOW)
    J.load_library().deflator_setdctnr(d._p, text[:50000], 50000)
    out = d.compress(text[50000:], chunk=10000, tgt=5000)
    d.close()
    assert out == oracle.deflate_dict(text[:50000], text[50000:], level=6)
    # default (independent-block) mode rejects a dictionary as misuse
    d = J.Deflator(6)
    J.load_library().deflator_setdctnr(d._p, b"abcd", 4)
    assert d.public.state == 0xDEADBEEF and d.public.error == J.engine.DEFLT_EINCORRECTUSE
    d.close()


def test_dropin_inflator_dictionary(engine, oracle):
    """inflator_setdctnr (inflator.c:905-925): references into the preset
    dictionary decode; streams from the oracle and from zlib's zdict."""
    J = engine
    text = J.corpus_text(300000, seed=43).tobytes()
    L = J.load_library()
    for dsize in (10, 5000, 32768, 50000):
        dic, data = text[:dsize], text[dsize:dsize + 120000]
        co = zlib.compressobj(9, zlib.DEFLATED, -15, zdict=dic[-32768:])
        for comp in (oracle.deflate_dict(dic, data, level=6), co.compress(data) + co.flush()):
            inf = J.Inflator()
            L.inflator_setdctnr(inf._p, dic, len(dic))
            out, r, e = inf.decompress(comp, chunk=7000, tgt=50000)
            inf.close()
            assert out == data and e == 0, (dsize, r, e)
    # without the dictionary the stream reaches too far back
    inf = J.Inflator()
    out, r, e = inf.decompress(oracle.deflate_dict(text[:5000], text[5000:60000], level=6))
    inf.close()
    assert r == J.engine.INFLT_ERROR and e == J.engine.INFLT_EFAROFFSET
    # a dictionary after use is misuse
    inf = J.Inflator()
    inf.decompress(oracle.deflate(b"hello"))
    L.inflator_setdctnr(inf._p, b"abc", 3)
    assert inf.public.state == 0xDEADBEEF and inf.public.error == J.engine.INFLT_EINCORRECTUSE
    inf.close()

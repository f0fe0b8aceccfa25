"""Parallel decode of streams without sync markers (k_fsp_find /
k_fsp_decode / k_fsp_window / k_fsp_resolve behind jdgpu_istream_inflate):
zlib's default output, Z_SYNC_FLUSH at arbitrary points, stored runs, preset
dictionaries.  The bar is the serial decoder's result bit for bit -- output,
status, error code and the bytes consumed -- with the parallel rounds
actually taken (their counters), and zlib's own decode for valid streams.
GPU tests, through the C ABI."""
import zlib

import numpy as np
import pytest

from jdeflate_amd import engine as E

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def zraw(data, level=6, zdict=None, sync_every=None, seed=0):
    kw = {"zdict": zdict} if zdict else {}
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 9, zlib.Z_DEFAULT_STRATEGY, **kw)
    if not sync_every:
        return c.compress(data) + c.flush()
    rng = np.random.default_rng(seed)
    out, i = [], 0
    while i < len(data):
        n = int(rng.integers(sync_every // 2, sync_every * 3 // 2))
        out.append(c.compress(data[i:i + n]))
        out.append(c.flush(zlib.Z_SYNC_FLUSH))
        i += n
    out.append(c.flush())
    return b"".join(out)


def decode(comp, cap, fsp=True, dict_=None, piece=None):
    """feed comp (whole, or in pieces) to one IStream; -> (out, statuses,
    last error, consumed total, fsp rounds, fsp chunks)"""
    s = E.IStream(dict_)
    s.fsp(1 if fsp else 0)
    out, sts, err, cons = [], [], 0, 0
    pos = 0
    piece = piece or max(len(comp), 1)
    while True:
        src = comp[pos:pos + piece]
        st, err, prod, used, _ = s.inflate(src, cap)
        out.append(s.out.raw[:prod])
        sts.append(st)
        cons += used
        pos += used
        if st in (E.IS_ENDED, E.IS_ERROR):
            break
        if st == E.IS_NEEDINPUT and pos >= len(comp):
            break
    rounds, chunks = s.fsp()
    s.close()
    return b"".join(out), sts, err, cons, rounds, chunks


@pytest.fixture(scope="module")
def text(engine):
    return engine.corpus_text(24 * MiB, seed=21).tobytes()


@pytest.mark.parametrize("level", [1, 6, 9])
def test_zlib_default_stream(text, level):
    comp = zraw(text, level)
    out, sts, err, cons, rounds, chunks = decode(comp, len(text) + 1)
    assert out == text
    assert sts[-1] == E.IS_ENDED and cons == len(comp)
    assert rounds >= 1 and chunks >= 8, (rounds, chunks)


def test_matches_serial(text):
    data = text[:6 * MiB]
    comp = zraw(data, 6)
    a = decode(comp, len(data) + 1)
    b = decode(comp, len(data) + 1, fsp=False)
    assert a[0] == b[0] == data
    assert a[1:4] == b[1:4]
    assert a[4] >= 1 and b[4] == 0


def test_sync_flush_points(text):
    data = text[:12 * MiB]
    comp = zraw(data, 6, sync_every=300_000, seed=3)
    out, sts, err, cons, rounds, chunks = decode(comp, len(data) + 1)
    assert out == data and sts[-1] == E.IS_ENDED and cons == len(comp)
    assert rounds >= 1


def test_mixed_with_stored_runs(engine, text):
    rng = np.random.default_rng(4)
    parts = []
    for i in range(24):
        parts.append(text[i * 400_000:(i + 1) * 400_000])
        if i % 5 == 2:
            parts.append(rng.integers(0, 256, 150_000, dtype=np.uint8).tobytes())
    data = b"".join(parts)
    comp = zraw(data, 6)
    out, sts, err, cons, rounds, chunks = decode(comp, len(data) + 1)
    assert out == data and sts[-1] == E.IS_ENDED and cons == len(comp)
    assert rounds >= 1


def test_preset_dictionary(text):
    zd = text[-40_000:]
    data = text[:8 * MiB]
    comp = zraw(data, 6, zdict=zd)
    out, sts, _, cons, rounds, _ = decode(comp, len(data) + 1, dict_=zd)
    assert out == data and sts[-1] == E.IS_ENDED and cons == len(comp)
    assert rounds >= 1


@pytest.mark.parametrize("piece,cap", [(3 * MiB + 17, 64 * MiB), (8 * MiB, 700_001)])
def test_pieces_and_small_targets(text, piece, cap):
    data = text[:16 * MiB]
    comp = zraw(data, 6)
    a = decode(comp, cap, piece=piece)
    assert a[0] == data and a[1][-1] == E.IS_ENDED and a[3] == len(comp)
    assert a[4] >= 1


@pytest.mark.parametrize("where", [0.3, 0.77])
def test_corrupt_stream_as_serial(text, oracle, where):
    """a flipped byte mid-stream: the parallel rounds accept only what the
    serial decode reaches, so the error and every delivered byte agree"""
    data = text[:6 * MiB]
    comp = bytearray(zraw(data, 6))
    k = int(len(comp) * where)
    comp[k] ^= 0x5A
    comp = bytes(comp)
    a = decode(comp, len(data) + 1)
    b = decode(comp, len(data) + 1, fsp=False)
    assert a[1:4] == b[1:4]
    assert a[0] == b[0]
    r, err, ref, _ = oracle.inflate(comp, 4 * len(data))
    if r == 0:
        assert a[1][-1] == E.IS_ENDED and a[0] == ref
    elif err == 6:
        assert a[1][-1] == E.IS_NEEDINPUT
    else:
        assert a[1][-1] == E.IS_ERROR and a[2] == err


def test_truncated_stream(text):
    data = text[:6 * MiB]
    comp = zraw(data, 6)
    cut = comp[:len(comp) * 2 // 3]
    a = decode(cut, len(data) + 1)
    b = decode(cut, len(data) + 1, fsp=False)
    assert a[0] == b[0] and a[1:4] == b[1:4]
    assert a[1][-1] == E.IS_NEEDINPUT
    assert data.startswith(a[0]) and len(a[0]) > 2 * MiB


def _logs(n):
    parts, i, size = [], 0, 0
    while size < n:
        s = "".join(f"2026-10-17 12:{(i + k) // 600 % 60:02d} host{(i + k) % 2} "
                    f"GET /api/v1/item/{(i + k) % 20} 200 {(i + k) % 7}ms\n" for k in range(1000))
        parts.append(s)
        size += len(s)
        i += 1000
    return "".join(parts).encode()[:n]


def test_high_ratio_stream_grows_chunk_room():
    """log-like data (ratio > 16, deflate blocks of megabytes): the first
    round's chunks run out of output entries, the next rounds get 4x the room
    per chunk (fewer chunks); output and result as zlib's"""
    data = _logs(128 * MiB)
    comp = zraw(data, 6)
    ratio = len(data) / len(comp)
    assert ratio > 16, ratio
    a = decode(comp, len(data) + 1)
    assert a[0] == data, "output differs"
    assert a[1][-1] == E.IS_ENDED and a[3] == len(comp)
    assert a[4] >= 2 and a[5] >= 8, a[4:]


def test_garbage_after_stream(text):
    """the final block ends the stream: search regions past it (random bytes
    behind the stream) are never accepted, and `consumed` stops exactly at
    the stream's last byte"""
    data = text[:8 * MiB]
    comp = zraw(data, 6)
    junk = np.random.default_rng(9).integers(0, 256, 3 * MiB, dtype=np.uint8).tobytes()
    a = decode(comp + junk, len(data) + 1)
    assert a[0] == data and a[1][-1] == E.IS_ENDED and a[3] == len(comp)
    assert a[4] >= 1


def test_random_data_stream(engine):
    """zlib on incompressible bytes: stored blocks and flat-coded Huffman
    blocks, where random bits pass header checks most often"""
    data = np.random.default_rng(10).integers(0, 256, 6 * MiB, dtype=np.uint8).tobytes()
    for level in (1, 9):
        comp = zraw(data, level)
        a = decode(comp, len(data) + 1)
        b = decode(comp, len(data) + 1, fsp=False)
        assert a[0] == data and a[1:4] == b[1:4]

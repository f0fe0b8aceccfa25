"""Single-window streams fed call by call: the drop-in
deflator with DEFLT_SINGLEWINDOW driven with a sequence of deflator_deflate
calls -- input in pieces without a flush, mid-stream DEFLT_FLUSH that keeps
the window (deflator.c:763-768), then DEFLT_END -- must write exactly what
the reference writes for the same calls: the oracle's call-sequence model
(oracle/jdoracle.c jdo_deflate_calls, deflator_deflate :691-786 per call).
GPU tests, through the C ABI."""
import random
import zlib

import pytest

from jdeflate_amd import engine as E

pytestmark = pytest.mark.gpu

NOF, END, FL = 0, 1, 2


def inflate_raw(b):
    return zlib.decompressobj(-15).decompress(b)


def check(oracle, data, calls, level, dictionary=b"", flags=0, tgt=1 << 20):
    want = oracle.deflate_calls(data, calls, level, flags, dictionary)
    got = E.deflate_calls(data, calls, level, flags, dictionary, tgt=tgt)
    assert len(got) == len(want) and got == want, (level, len(got), len(want), calls[:6])
    if dictionary:
        d = zlib.decompressobj(-15, zdict=dictionary[-32768:])
        assert d.decompress(got) == data
    else:
        assert inflate_raw(got) == data


@pytest.fixture(scope="module")
def corpora(engine):
    J = engine
    text = J.corpus_text(1_200_000, seed=41).tobytes()
    mixed = J.corpus_mixed(700_000, seed=42).tobytes()
    return {"text": text, "mixed": mixed}


def flush_every(n, step, first=None):
    ends = list(range(first or step, n, step))
    return [(e, FL) for e in ends] + [(n, END)]


@pytest.mark.parametrize("level", [1, 3, 6, 9])
def test_flush_every_100k(engine, oracle, corpora, level):
    data = corpora["text"][:700_000]
    check(oracle, data, flush_every(len(data), 100_000), level)


@pytest.mark.parametrize("level", [0, 6])
def test_flush_points_mixed(engine, oracle, corpora, level):
    data = corpora["mixed"][:500_000]
    calls = [(1, FL), (2, FL), (5, FL), (70_000, FL), (70_003, FL), (200_000, FL),
             (200_000, FL), (333_333, FL), (len(data), END)]
    check(oracle, data, calls, level)


def test_short_flushes_accumulate(engine, oracle, corpora):
    """many flush points within the carried history: the stale buckets of
    each stay in force"""
    data = corpora["text"][:120_000]
    rnd = random.Random(5)
    ends = sorted(set(rnd.randrange(1, len(data)) for _ in range(40)))
    calls = [(e, FL) for e in ends] + [(len(data), END)]
    check(oracle, data, calls, 6)
    check(oracle, data, calls, 9)


def test_long_stream_trims_history(engine, oracle, corpora):
    """1.2 MB with flushes every 150-250 KB: the history moves on, the hash-3
    heads are carried from the previous piece's scan"""
    data = corpora["text"]
    rnd = random.Random(7)
    ends, e = [], 0
    while True:
        e += rnd.randrange(150_000, 250_000)
        if e >= len(data):
            break
        ends.append(e)
    calls = [(x, FL) for x in ends] + [(len(data), END)]
    check(oracle, data, calls, 6)


@pytest.mark.parametrize("level", [2, 6, 9])
def test_noflush_pieces_then_end(engine, oracle, corpora, level):
    """input in pieces without a flush: the reference's window fills at the
    call ends (fillwindow with the call's remaining source)"""
    data = corpora["text"][:600_000]
    rnd = random.Random(level)
    ends, e = [], 0
    while True:
        e += rnd.choice([rnd.randrange(1, 3000), rnd.randrange(3000, 140_000), 131072 - rnd.randrange(1, 1023)])
        if e >= len(data):
            break
        ends.append(e)
    calls = [(x, NOF) for x in ends] + [(len(data), END)]
    check(oracle, data, calls, level)


def test_noflush_and_flush_mixed(engine, oracle, corpora):
    data = corpora["mixed"][:400_000]
    calls = [(10_000, NOF), (130_000, NOF), (131_000, FL), (131_500, NOF), (260_000, NOF),
             (262_000, FL), (262_000, NOF), (300_000, FL), (len(data), END)]
    check(oracle, data, calls, 6)
    check(oracle, data, calls, 9)


def test_dictionary_then_flushes(engine, oracle, corpora):
    d = corpora["text"][-40_000:]
    data = corpora["text"][:300_000]
    calls = [(3, FL), (50_000, FL), (50_001, NOF), (180_000, FL), (len(data), END)]
    check(oracle, data, calls, 6, dictionary=d)
    check(oracle, data, calls, 4, dictionary=d)


def test_small_targets(engine, oracle, corpora):
    data = corpora["text"][:200_000]
    check(oracle, data, flush_every(len(data), 30_000), 6, tgt=777)


def test_flush_then_end_empty(engine, oracle, corpora):
    data = corpora["text"][:50_000]
    check(oracle, data, [(len(data), FL), (len(data), END)], 6)
    check(oracle, b"", [(0, FL), (0, FL), (0, END)], 6)
    check(oracle, data[:10], [(10, FL), (10, END)], 9)


def test_chunkings_against_model(engine, oracle, corpora):
    """random call sequences near the window size, where a slide can happen
    with the window not yet full (a generation's bytes then show past the
    end)"""
    base = corpora["text"]
    rnd = random.Random(11)
    for trial in range(6):
        n = rnd.randrange(140_000, 420_000)
        data = base[:n - 3000] + base[n - 9000:n - 6000]
        ends, e = [], rnd.randrange(1000, 140_000)
        while e < len(data):
            ends.append(e)
            e += rnd.choice([rnd.randrange(1, 2000), rnd.randrange(1000, 131072),
                             131072 - rnd.randrange(1, 1023)])
        calls = [(x, rnd.choice([NOF, NOF, NOF, FL])) for x in ends] + [(len(data), END)]
        check(oracle, data, calls, rnd.choice([6, 9, 3]))


def test_held_step_across_block_accepts(engine, oracle):
    """a match held at a 64 KiB block's last position and replaced by an
    accept at the next block's first: the literal's entry starts at -1 of
    that block (corpus seed 41: positions 327679 and 655359; the accepted
    offset >= 16384 once set bit 31 of the unmasked token)"""
    data = engine.corpus_text(700_000, seed=41).tobytes()
    assert E.deflate_stream(data, 6) == oracle.deflate(data, 6)

"""The CPU restatement (oracle) against the reference's known answers, the
golden fixtures and RFC 1951 (Python zlib).  No GPU."""
import hashlib
import json
import os
import zlib

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def c1_input():
    s = b"The quick brown fox jumps over the lazy dog. "
    return (s * (1048576 // len(s) + 1))[:1048576]


def test_known_answer_c1_single_stream(oracle):
    # the reference writes 3,117 bytes
    out = oracle.deflate(c1_input(), level=6, flush=1)
    assert len(out) == 3117
    assert zlib.decompressobj(-15).decompress(out) == c1_input()


def test_known_answer_position0_quirk(oracle):
    # literal at position 10, length-9 match at 11
    t = oracle.trace(b"ABCDEFGHIJABCDEFGHIJ", level=6)
    lits = [x for x in t[:11]]
    assert lits == list(b"ABCDEFGHIJA")
    assert t[11] == 0x80000000 | (9 << 16) | 10


def test_known_answer_random_block_split(oracle):
    # 65,533 slots then a static remainder
    data = np.random.default_rng(1).integers(0, 256, 65536, dtype=np.uint8).tobytes()
    t = oracle.trace(data, level=6)
    ends = [i for i, x in enumerate(t) if x & 0x40000000 and not x & 0x80000000]
    assert len(ends) == 2
    first = t[:ends[0]]
    slots = sum(3 if x & 0x80000000 else 1 for x in first)
    assert slots + 4 > 65536 >= slots + 1
    assert t[ends[0]] == 0x40000002 and t[ends[1]] == 0x40000001


def test_golden_fixtures(oracle):
    man = json.load(open(os.path.join(GOLD, "manifest.json")))
    assert len(man["cases"]) >= 100
    for c in man["cases"]:
        data = open(os.path.join(GOLD, c["input"]), "rb").read()
        assert hashlib.sha256(data).hexdigest() == c["in_sha256"]
        out = oracle.deflate(data, level=c["level"], flush=1 if c["flush"] == "end" else 2)
        assert hashlib.sha256(out).hexdigest() == c["out_sha256"], c
        assert out == open(os.path.join(GOLD, c["output"]), "rb").read()
        # independent RFC 1951 decoder
        assert zlib.decompressobj(-15).decompress(out) == data


@pytest.mark.parametrize("level", range(10))
def test_zlib_round_trip_all_levels(oracle, level):
    rng = np.random.default_rng(level)
    inputs = [b"", b"x", bytes(70000), rng.integers(0, 256, 70000, dtype=np.uint8).tobytes(),
              rng.integers(0, 3, 150000, dtype=np.uint8).tobytes(),
              open(os.__file__, "rb").read()]
    for data in inputs:
        for flush in (1, 2):
            out = oracle.deflate(data, level=level, flush=flush)
            assert zlib.decompressobj(-15).decompress(out) == data


def test_flush_joined_blocks_are_one_stream(oracle):
    # fresh-state FLUSH blocks + END concatenate into one stream
    data = np.random.default_rng(3).integers(0, 4, 300000, dtype=np.uint8).tobytes()
    out, sizes = oracle.deflate_blocks(data, level=6)
    assert sum(sizes) == len(out) and len(sizes) == 5
    assert zlib.decompressobj(-15).decompress(out) == data
    back, us, er = oracle.inflate_blocks(out, sizes)
    assert back == data and not any(er)


def test_levels_differ_on_text(oracle):
    import jdeflate_amd as J
    try:
        t = J.corpus_text(4 * 65536, seed=9).tobytes()
    except Exception:
        pytest.skip("corpus helper not built")
    sizes = [len(oracle.deflate_blocks(t, level=lv)[0]) for lv in (1, 6, 9)]
    assert sizes[0] > sizes[1] > sizes[2]


@pytest.mark.parametrize("strategy", [0, 1, 2, 3, 4])
def test_inflate_zlib_streams(oracle, strategy):
    data = open(os.__file__, "rb").read() * 3
    for level in (1, 6, 9):
        co = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
        c = co.compress(data) + co.flush()
        r, e, out, cons = oracle.inflate(c, len(data))
        assert r == 0 and e == 0 and out == data and cons == len(c)


def _dynamic_header(hlit, hdist, hclen):
    v = 0b10 << 1 | 1                 # BFINAL=1, BTYPE=2
    v |= (hlit - 257) << 3 | (hdist - 1) << 8 | (hclen - 4) << 13
    return v.to_bytes(3, "little")


def test_inflate_error_codes(oracle):
    cap = 1 << 16
    assert oracle.inflate(b"", cap)[:2] == (3, 6)                   # EINPUTEND
    assert oracle.inflate(b"\x07", cap)[:2] == (3, 5)               # BTYPE 3: EBADBLOCK
    assert oracle.inflate(b"\x01\x05\x00\x00\x00abcde", cap)[:2] == (3, 5)  # LEN/NLEN
    assert oracle.inflate(_dynamic_header(287, 1, 4), cap)[:2] == (3, 3)    # HLIT > 286
    good = zlib.compressobj(6, zlib.DEFLATED, -15)
    c = good.compress(b"hello hello hello hello") + good.flush()
    assert oracle.inflate(c[:-2], cap)[:2] == (3, 6)                 # truncated
    # static block: literal 'a', then length 3 at distance 5 (> 1 byte out)
    assert oracle.inflate(static_block([("lit", ord("a")), ("match", 3, 5)]), cap)[:2] == (3, 4)


def static_block(items, final=1):
    """Hand-assemble a fixed-Huffman block (RFC 1951 3.2.6)."""
    acc, nb = 0, 0

    def put(v, n):
        nonlocal acc, nb
        acc |= v << nb
        nb += n

    def code(c, n):
        put(int(format(c, f"0{n}b")[::-1], 2), n)

    def lit(s):
        if s < 144:
            code(0x30 + s, 8)
        elif s < 256:
            code(0x190 + s - 144, 9)
        elif s < 280:
            code(s - 256, 7)
        else:
            code(0xC0 + s - 280, 8)

    put(final, 1)
    put(1, 2)
    lb = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83,
          99, 115, 131, 163, 195, 227, 258]
    le = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
    db = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025,
          1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577]
    de = [0, 0, 0, 0] + [i // 2 for i in range(2, 28)]
    for it in items:
        if it[0] == "lit":
            lit(it[1])
        else:
            ln, d = it[1], it[2]
            s = max(i for i in range(29) if lb[i] <= ln)
            lit(257 + s)
            put(ln - lb[s], le[s])
            k = max(i for i in range(30) if db[i] <= d)
            code(k, 5)
            put(d - db[k], de[k])
    lit(256)
    return acc.to_bytes((nb + 7) // 8, "little")


def test_static_block_helper_round_trips(oracle):
    raw = static_block([("lit", ord("x")), ("lit", ord("y")), ("match", 10, 2)])
    assert zlib.decompressobj(-15).decompress(raw) == b"xy" * 6
    r, e, out, _ = oracle.inflate(raw, 100)
    assert (r, e, out) == (0, 0, b"xy" * 6)

"""GPU parity: the HIP engine against the oracle (bit-exact), through the
C ABI.  Sizes here are small enough for the oracle; the full-size test uses
size-independent properties plus a multi-threaded oracle comparison."""
import ctypes
import json
import os
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BS = 65536


def corpora(J):
    rng = np.random.default_rng(11)
    return {
        "text": J.corpus_text(5 * BS + 4321, seed=21).tobytes(),
        "mixed": J.corpus_mixed(20 * BS, seed=22).tobytes(),
        "random": rng.integers(0, 256, 2 * BS + 77, dtype=np.uint8).tobytes(),
        "zeros": bytes(3 * BS + 5),
        "runs": bytes(np.repeat(rng.choice([0, 1, 255], 3000),
                                rng.integers(1, 120, 3000)).astype(np.uint8)),
        "src": open(os.__file__, "rb").read() * 2,
    }


@pytest.mark.parametrize("level", [6, 9, 7, 8, 1, 2, 3, 4, 5, 0])
def test_deflate_parity_all_levels(engine, oracle, level):
    for name, data in corpora(engine).items():
        g, gs = engine.deflate_blocks(data, level=level)
        r, rs = oracle.deflate_blocks(data, level=level)
        assert gs == rs, (name, level)
        assert g == r, (name, level)
        assert zlib.decompressobj(-15).decompress(g) == data


@pytest.mark.parametrize("level", [6, 7, 8, 9])
def test_split_parse_equals_oracle(engine, oracle, level):
    """Levels 6-9 parse with the segment-split k_pspec/k_psync/k_pjoin.  It
    must give the reference's bytes, including data whose doshort flag flips
    often (bytes < 16 as literals) and data where segment walks meet late or
    not at all."""
    rng = np.random.default_rng(level)
    words = [bytes(rng.integers(0, 24, rng.integers(1, 7), dtype=np.uint8)) for _ in range(300)]
    low = b"".join(words[i] for i in rng.integers(0, 300, 60000))[:9 * BS + 321]
    # > 16 blocks of every k_pweight class, interleaved (incompressible,
    # long runs, text, zeros, low bytes): k_porder's class-sorted walk order
    # and the block join's doshort-stop staging both run on purpose
    kinds = []
    for i in range(25):
        k = i % 5
        if k == 0:
            kinds.append(rng.integers(0, 256, BS, dtype=np.uint8).tobytes())
        elif k == 1:
            kinds.append(bytes(np.repeat(rng.choice([0, 1, 255], 2000),
                                         rng.integers(8, 200, 2000)).astype(np.uint8))[:BS])
        elif k == 2:
            kinds.append(engine.corpus_text(BS, seed=500 + i).tobytes())
        elif k == 3:
            kinds.append(bytes(BS))
        else:
            kinds.append(low[(i * 4099) % (len(low) - BS):][:BS])
    data = {"low": low, "mixed": engine.corpus_mixed(24 * BS, seed=40 + level).tobytes(),
            "text": engine.corpus_text(6 * BS + 99, seed=level).tobytes(),
            "classes": b"".join(kinds)}
    for name, d in data.items():
        r, rs = oracle.deflate_blocks(d, level=level)
        g, gs = engine.deflate_blocks(d, level=level)
        assert (g, gs) == (r, rs), (name, level)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 5, 258, 259, 262, 4095, 65535, 65536, 65537,
                               2 * BS + 17])
def test_edge_sizes(engine, oracle, n):
    data = engine.corpus_text(max(n, 1), seed=n + 1).tobytes()[:n]
    for level in (0, 1, 6, 9):
        g, gs = engine.deflate_blocks(data, level=level)
        r, rs = oracle.deflate_blocks(data, level=level)
        assert (g, gs) == (r, rs), (n, level)
        back, us, er = engine.inflate_blocks(g, gs)
        assert back == data and not any(er)


def test_golden_fixtures(engine):
    man = json.load(open(os.path.join(GOLD, "manifest.json")))
    for c in man["cases"]:
        data = open(os.path.join(GOLD, c["input"]), "rb").read()
        want = open(os.path.join(GOLD, c["output"]), "rb").read()
        flush = 1 if c["flush"] == "end" else 2
        got, sizes = engine.deflate_blocks(data, level=c["level"], lastflush=flush)
        assert got == want, c
        back, us, er = engine.inflate_blocks(got, sizes)
        assert back == data and not any(er), c


@pytest.mark.parametrize("bs", [16, 4096, 16384, 32768])
def test_other_block_sizes(engine, oracle, bs):
    data = engine.corpus_mixed(6 * BS, seed=bs, blocksize=BS).tobytes()[:5 * BS + 1000]
    for level in (1, 6, 9):
        g, gs = engine.deflate_blocks(data, level=level, blocksize=bs)
        r, rs = oracle.deflate_blocks(data, level=level, blocksize=bs)
        assert (g, gs) == (r, rs), (bs, level)
        back, _, er = engine.inflate_blocks(g, gs, blocksize=bs)
        assert back == data and not any(er)


def test_many_chunks(engine, oracle):
    # more blocks than one launch chunk (16384) exercises the device-side
    # offset carry between chunks
    bs = 16
    data = engine.corpus_text(16400 * bs + 5, seed=5).tobytes()
    g, gs = engine.deflate_blocks(data, level=6, blocksize=bs)
    r, rs = oracle.deflate_blocks(data, level=6, blocksize=bs)
    assert (g, gs) == (r, rs)


def test_fixed_codes_flag(engine, oracle):
    data = engine.corpus_text(3 * BS, seed=8).tobytes()
    for level in (2, 6, 9):
        g, gs = engine.deflate_blocks(data, level=level, flags=1)
        r, rs = oracle.deflate_blocks(data, level=level, flags=1)
        assert (g, gs) == (r, rs)


def test_flush_last_block(engine, oracle):
    data = engine.corpus_text(BS + 100, seed=3).tobytes()
    g, gs = engine.deflate_blocks(data, level=6, lastflush=2)
    r = oracle.deflate(data[:BS], level=6, flush=2) + oracle.deflate(data[BS:], level=6, flush=2)
    assert g == r


def test_inflate_zlib_single_streams(engine):
    data = open(os.__file__, "rb").read() * 4
    for level in (0, 1, 6, 9):
        for strategy in (0, 1, 2, 3, 4):
            co = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
            c = co.compress(data) + co.flush()
            out, err, used = engine.inflate_stream(c, len(data) + 16)
            assert err == 0 and out == data and used == len(c), (level, strategy)


def test_inflate_corrupt_blocks_match_oracle(engine, oracle):
    data = engine.corpus_text(8 * BS, seed=31).tobytes()
    g, gs = engine.deflate_blocks(data, level=6)
    rng = np.random.default_rng(7)
    raw = bytearray(g)
    offs = np.cumsum([0] + gs[:-1])
    for i in range(len(gs)):            # one flipped bit per block
        pos = int(offs[i] + rng.integers(0, gs[i] - 4))
        raw[pos] ^= 1 << int(rng.integers(0, 8))
    bad = bytes(raw)
    gout, gus, ger = engine.inflate_blocks(bad, gs)
    oout, ous, oer = oracle.inflate_blocks(bad, gs)
    assert ger == oer
    assert gus == ous
    assert gout == oout


def test_inflate_blocks_made_by_zlib(engine, oracle):
    """Block-mode inflate of independent blocks compressed by zlib (every
    strategy: dynamic, fixed-Huffman, RLE, stored at level 0, filtered),
    FLUSH-terminated like the reference's blocks -- exercises the lane
    decoder on trees and block mixes our encoder never emits."""
    rng = np.random.default_rng(17)
    texts = engine.corpus_mixed(24 * BS, seed=43).tobytes()
    blocks, want = [], []
    for i in range(24):
        blk = texts[i * BS:(i + 1) * BS]
        if i % 6 == 5:
            blk = bytes(rng.integers(0, 256, BS, dtype=np.uint8))
        level = [0, 1, 6, 9][i % 4]
        strategy = [0, 1, 2, 3, 4][i % 5]
        co = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
        blocks.append(co.compress(blk) + co.flush(zlib.Z_SYNC_FLUSH))
        want.append(blk)
    sizes = [len(b) for b in blocks]
    g = b"".join(blocks)
    out, us, er = engine.inflate_blocks(g, sizes)
    oout, ous, oer = oracle.inflate_blocks(g, sizes)
    assert (out, us, er) == (oout, ous, oer)
    assert out == b"".join(want) and not any(er)


def _kind_blocks(rng, kinds):
    """64 KiB blocks of the mixed corpus' record-heavy kinds: int32 ramps plus
    noise (a dense list of short, chained copies), runs over {0, 1, 255}, zeros
    (long chained copies), and text between them"""
    out = []
    for k in kinds:
        if k == "ramps":
            a, step = np.uint64(rng.integers(0, 1 << 32)), np.uint64(rng.integers(1, 1000))
            v = a + np.arange(BS // 4, dtype=np.uint64) * step + rng.integers(0, 16, BS // 4).astype(np.uint64)
            out.append((v & np.uint64(0xffffffff)).astype("<u4").tobytes())
        elif k == "runs":
            b = bytearray()
            while len(b) < BS:
                b += bytes([int(rng.choice([0, 1, 255]))]) * int(rng.integers(1, 201))
            out.append(bytes(b[:BS]))
        elif k == "zero":
            out.append(bytes(BS))
        else:
            out.append(None)
    return out


@pytest.mark.parametrize("level", [6, 9])
def test_inflate_fused_resolve_kinds(engine, oracle, level):
    """k_inflate_par resolves the records of dense or long-record blocks itself
    (ramps, runs, zeros) and leaves the rest to k_inflate_resolve: a launch
    mixing both kinds of block, clean and with a flipped bit in a fused one,
    decodes exactly as the oracle does."""
    rng = np.random.default_rng(61 + level)
    kinds = ["ramps", "text", "runs", "zero", "ramps", "text", "runs", "ramps", "zero", "text"] * 2
    blocks = _kind_blocks(rng, kinds)
    text = engine.corpus_text(len(kinds) * BS, seed=62).tobytes()
    data = b"".join(b if b is not None else text[i * BS:(i + 1) * BS] for i, b in enumerate(blocks))
    g, gs = engine.deflate_blocks(data, level=level)
    back, us, er = engine.inflate_blocks(g, gs)
    assert back == data and not any(er)
    raw = bytearray(g)
    offs = np.cumsum([0] + gs[:-1])
    raw[int(offs[4]) + gs[4] // 2] ^= 0x08          # inside a ramps block
    raw[int(offs[2]) + gs[2] // 2] ^= 0x40          # inside a runs block
    bad = bytes(raw)
    gout, gus, ger = engine.inflate_blocks(bad, gs)
    oout, ous, oer = oracle.inflate_blocks(bad, gs)
    assert (gout, gus, ger) == (oout, ous, oer)


def test_inflate_fallback_path(engine, oracle, monkeypatch):
    """Blocks whose record list exceeds the per-lane budget are decoded by
    the wave-per-block kernel; with the budget forced tiny most blocks take
    that route (mixed with lane-decoded ones), results stay bit-exact --
    including corrupt blocks."""
    data = engine.corpus_mixed(12 * BS, seed=41).tobytes() + engine.corpus_text(9 * BS + 77, seed=42).tobytes()
    g, gs = engine.deflate_blocks(data, level=6)
    raw = bytearray(g)
    offs = np.cumsum([0] + gs[:-1])
    raw[int(offs[3]) + 40] ^= 0x10
    bad = bytes(raw)
    for cap in ("3", "200", "5000"):
        monkeypatch.setenv("JD_INFLATE_RECCAP", cap)
        back, us, er = engine.inflate_blocks(g, gs)
        assert back == data and not any(er), cap
        gout, gus, ger = engine.inflate_blocks(bad, gs)
        oout, ous, oer = oracle.inflate_blocks(bad, gs)
        assert (gout, gus, ger) == (oout, ous, oer), cap


def test_inflate_error_codes_match_oracle(engine, oracle):
    cases = [b"\x07", b"\x01\x05\x00\x00\x00abcde", bytes([0xff, 0xff, 0xff]),
             b"\x0b\x00", b"\x05\x00\x00\x00"]
    for c in cases:
        out, err, _ = engine.inflate_stream(c, 1 << 16)
        r, e, o, _ = oracle.inflate(c, 1 << 16)
        assert err == e, (c, err, e)
        assert out == o


def test_dropin_deflator_streaming(engine, oracle):
    data = engine.corpus_text(3 * BS + 999, seed=12).tobytes()
    want, _ = oracle.deflate_blocks(data, level=6)
    for chunk, tgt in ((1 << 30, 1 << 20), (7, 13), (BS, 100), (1000, 65536)):
        d = engine.Deflator(6)
        assert d.compress(data, chunk=chunk, tgt=tgt) == want, (chunk, tgt)
        d.close()


def test_dropin_deflator_misuse_and_reset(engine):
    J = engine
    d = J.Deflator(6)
    d.setsrc(b"abc")
    d.settgt(100)
    assert d.deflate(J.DEFLT_NOFLUSH) == J.engine.DEFLT_SRCEXHSTD
    # no new source after SRCEXHSTD and no flush: EINCORRECTUSE (validate :671-679)
    assert d.deflate(J.DEFLT_NOFLUSH) == J.engine.DEFLT_ERROR
    assert d.public.error == J.engine.DEFLT_EINCORRECTUSE
    assert d.deflate(J.DEFLT_END) == J.engine.DEFLT_ERROR          # poisoned
    d.reset()
    out = d.compress(b"hello")
    assert zlib.decompressobj(-15).decompress(out) == b"hello"
    d.close()


def test_dropin_deflator_sync_flush(engine, oracle):
    J = engine
    a = J.corpus_text(70000, seed=1).tobytes()
    b = J.corpus_text(5000, seed=2).tobytes()
    d = J.Deflator(6)
    part1 = d.compress(a, flush=J.DEFLT_FLUSH)
    part2 = d.compress(b, flush=J.DEFLT_END)
    want = (oracle.deflate(a[:BS], flush=2) + oracle.deflate(a[BS:], flush=2) +
            oracle.deflate(b, flush=1))
    assert part1 + part2 == want
    assert zlib.decompressobj(-15).decompress(part1 + part2) == a + b


def test_dropin_inflator(engine):
    J = engine
    data = J.corpus_text(2 * BS + 33, seed=4).tobytes()
    g, _ = J.deflate_blocks(data, level=6)
    for chunk, tgt in ((1 << 30, 1 << 20), (100, 7), (4096, 65536)):
        inf = J.Inflator()
        out, r, e = inf.decompress(g, chunk=chunk, tgt=tgt)
        assert (out, r, e) == (data, 0, 0)
        inf.close()
    co = zlib.compressobj(9, zlib.DEFLATED, -15)
    z = co.compress(data) + co.flush()
    inf = J.Inflator()
    assert inf.decompress(z, chunk=333, tgt=1000) == (data, 0, 0)
    inf.close()
    inf = J.Inflator()
    out, r, e = inf.decompress(z[:len(z) // 2])
    assert r == J.engine.INFLT_ERROR and e == J.engine.INFLT_EINPUTEND
    assert data.startswith(out)
    inf.close()


def test_device_api_torch(engine, oracle):
    import torch
    J = engine
    data = J.corpus_mixed(40 * BS, seed=77)
    n = data.size
    nb = n // BS
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(data).to(dev)
    cap = J.bound(n)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_csz = torch.empty(nb, dtype=torch.int32, device=dev)
    d_coff = torch.empty(nb, dtype=torch.int64, device=dev)
    d_tot = torch.zeros(1, dtype=torch.int64, device=dev)
    s = torch.cuda.Stream(dev)
    J.deflate_device(d_in.data_ptr(), n, d_out.data_ptr(), cap, d_csz.data_ptr(),
                     d_coff.data_ptr(), d_tot.data_ptr(), level=9, stream=s.cuda_stream)
    d_back = torch.empty(n, dtype=torch.uint8, device=dev)
    d_us = torch.empty(nb, dtype=torch.int32, device=dev)
    d_err = torch.empty(nb, dtype=torch.int32, device=dev)
    J.inflate_device(d_out.data_ptr(), cap, d_coff.data_ptr(), d_csz.data_ptr(), nb,
                     d_back.data_ptr(), d_us.data_ptr(), d_err.data_ptr(), stream=s.cuda_stream)
    s.synchronize()
    total = int(d_tot.item())
    r, rs = oracle.deflate_blocks(data.tobytes(), level=9)
    assert total == len(r)
    assert d_out[:total].cpu().numpy().tobytes() == r
    assert d_csz.cpu().numpy().tolist() == rs
    assert torch.equal(d_back, d_in) and int(d_err.abs().sum()) == 0


@pytest.mark.parametrize("nb", [1024, 1023])
def test_device_inflate_exact_output_buffer(engine, oracle, nb):
    """All-zero 64 KiB blocks end with a length-3 distance-1 match at byte
    65533, so the resolve copies a source at the output buffer's last bytes.
    The output tensor is exactly n bytes: no copy may read past it (this
    faulted when the resolve loaded the dword after every source)."""
    import torch
    J = engine
    n = nb * BS
    dev = torch.device("cuda", 0)
    one = oracle.deflate(bytes(BS), level=9, flush=2)
    last = oracle.deflate(bytes(BS), level=9, flush=1)
    comp = np.frombuffer(one * (nb - 1) + last, dtype=np.uint8).copy()
    d_c = torch.from_numpy(comp).to(dev)
    d_coff = torch.tensor([i * len(one) for i in range(nb)], dtype=torch.int64, device=dev)
    d_csz = torch.tensor([len(one)] * (nb - 1) + [len(last)], dtype=torch.int32, device=dev)
    d_back = torch.empty(n, dtype=torch.uint8, device=dev)
    d_us = torch.empty(nb, dtype=torch.int32, device=dev)
    d_err = torch.empty(nb, dtype=torch.int32, device=dev)
    J.inflate_device(d_c.data_ptr(), comp.size, d_coff.data_ptr(), d_csz.data_ptr(), nb,
                     d_back.data_ptr(), d_us.data_ptr(), d_err.data_ptr())
    torch.cuda.synchronize()
    assert int(d_err.abs().sum()) == 0 and bool((d_us == BS).all())
    assert not bool(d_back.any())
    # and the device deflate of the same blocks into an exact-size target
    d_in = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_out = torch.empty(J.bound(n), dtype=torch.uint8, device=dev)
    d_tot = torch.zeros(1, dtype=torch.int64, device=dev)
    J.deflate_device(d_in.data_ptr(), n, d_out.data_ptr(), d_out.numel(), d_csz.data_ptr(),
                     d_coff.data_ptr(), d_tot.data_ptr(), level=9)
    torch.cuda.synchronize()
    assert d_out[:int(d_tot.item())].cpu().numpy().tobytes() == comp.tobytes()


def test_full_size_round_trip_and_parity(engine, oracle):
    """1 GiB (configs C2/C3): GPU output equals the multi-threaded oracle's
    byte for byte, and inflates back to the input."""
    J = engine
    n = 1 << 30
    data = J.corpus_text(n, seed=1000, threads=16)
    g, gs = J.deflate_blocks(data.tobytes(), level=6)
    nb = n // BS
    L = oracle.lib()
    slot = L.jdo_bound(BS) + 64
    dst = np.empty(nb * slot, dtype=np.uint8)
    sizes = (ctypes.c_uint32 * nb)()
    L.jdo_deflate_blocks_mt(data.ctypes.data, n, BS, 6, dst.ctypes.data, slot, sizes, 16)
    assert list(sizes) == gs
    offs = np.concatenate([[0], np.cumsum(gs)])
    for i in range(0, nb, 97):          # byte-compare a spread of blocks
        o = int(offs[i])
        assert g[o:o + gs[i]] == dst[i * slot:i * slot + gs[i]].tobytes()
    back, us, er = J.inflate_blocks(g, gs)
    assert not any(er) and back == data.tobytes()


def test_level9_mixed_parity_128mib(engine, oracle):
    """configs[4]'s workload shape (Silesia-like mix, level 9) at 128 MiB:
    sizes of every block and the bytes of a spread of blocks equal the
    multi-threaded oracle's; the round trip is exact."""
    J = engine
    n = 128 << 20
    data = J.corpus_mixed(n, seed=2024, threads=16)
    g, gs = J.deflate_blocks(data.tobytes(), level=9)
    nb = n // BS
    L = oracle.lib()
    slot = L.jdo_bound(BS) + 64
    dst = np.empty(nb * slot, dtype=np.uint8)
    sizes = (ctypes.c_uint32 * nb)()
    L.jdo_deflate_blocks_mt(data.ctypes.data, n, BS, 9, dst.ctypes.data, slot, sizes, 16)
    assert list(sizes) == gs
    offs = np.concatenate([[0], np.cumsum(gs)])
    for i in range(0, nb, 13):
        o = int(offs[i])
        assert g[o:o + gs[i]] == dst[i * slot:i * slot + gs[i]].tobytes(), i
    back, us, er = J.inflate_blocks(g, gs)
    assert not any(er) and back == data.tobytes()


def _device_round_trip(J, data, level, lastflush=1):
    """deflate_device + inflate_device on HBM-resident data; returns
    (csizes, coffs, d_out, ok) with the round trip checked on the device"""
    import torch
    n = data.size
    nb = n // BS
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(data).to(dev)
    cap = J.bound(n)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_csz = torch.empty(nb, dtype=torch.int32, device=dev)
    d_coff = torch.empty(nb, dtype=torch.int64, device=dev)
    d_tot = torch.zeros(1, dtype=torch.int64, device=dev)
    s = torch.cuda.Stream(dev)
    J.deflate_device(d_in.data_ptr(), n, d_out.data_ptr(), cap, d_csz.data_ptr(),
                     d_coff.data_ptr(), d_tot.data_ptr(), level=level, lastflush=lastflush,
                     stream=s.cuda_stream)
    d_back = torch.empty(n, dtype=torch.uint8, device=dev)
    d_us = torch.empty(nb, dtype=torch.int32, device=dev)
    d_err = torch.empty(nb, dtype=torch.int32, device=dev)
    J.inflate_device(d_out.data_ptr(), cap, d_coff.data_ptr(), d_csz.data_ptr(), nb,
                     d_back.data_ptr(), d_us.data_ptr(), d_err.data_ptr(), stream=s.cuda_stream)
    s.synchronize()
    ok = bool(torch.equal(d_back, d_in)) and int(d_err.abs().sum()) == 0
    del d_back, d_in
    return (d_csz.cpu().numpy().astype(np.int64), d_coff.cpu().numpy(), d_out, ok,
            int(d_tot.item()))


def test_c5_level9_mixed_4gib(engine, oracle):
    """configs[4] at its stated size: 4 GiB Silesia-like mix, level 9, 65,536
    blocks (4 launch chunks, device-side offset carry).  Every block size
    equals the multi-threaded oracle's, a spread of blocks is byte-compared,
    the round trip is exact."""
    J = engine
    n = 4 << 30
    nb = n // BS
    data = J.corpus_mixed(n, seed=2025, threads=16)
    csz, coff, d_out, ok, total = _device_round_trip(J, data, 9)
    print(f"gpu done: {total} B, round trip {ok}", flush=True)
    assert ok
    L = oracle.lib()
    slot = L.jdo_bound(BS) + 64
    dst = np.empty(nb * slot, dtype=np.uint8)
    sizes = (ctypes.c_uint32 * nb)()
    L.jdo_deflate_blocks_mt(data.ctypes.data, n, BS, 9, dst.ctypes.data, slot, sizes, 16)
    ref = np.frombuffer(sizes, dtype=np.uint32).astype(np.int64)
    assert np.array_equal(ref, csz), int(np.flatnonzero(ref != csz)[0])
    assert total == int(ref.sum())
    for i in list(range(0, nb, 509)) + [nb - 1]:
        o = int(coff[i])
        got = d_out[o:o + int(csz[i])].cpu().numpy().tobytes()
        assert got == dst[i * slot:i * slot + int(csz[i])].tobytes(), i


def test_c4_shard_8gib_131072_blocks(engine, oracle):
    """One GPU's shard of configs[3] (64 GiB over 8 GPUs): 8 GiB, 131,072
    blocks (8 launch chunks), the shard ending with FLUSH as every rank but
    the last does.  Round trip exact; sizes and bytes of sampled blocks equal
    the oracle's."""
    J = engine
    n = 8 << 30
    nb = n // BS
    data = J.corpus_text(n, seed=4242, threads=16)
    csz, coff, d_out, ok, total = _device_round_trip(J, data, 6, lastflush=2)
    print(f"gpu done: {total} B, round trip {ok}", flush=True)
    assert ok and total == int(csz.sum())
    step = 61
    idx = np.arange(0, nb, step)
    sample = np.ascontiguousarray(data.reshape(nb, BS)[idx]).reshape(-1)
    L = oracle.lib()
    slot = L.jdo_bound(BS) + 64
    ns = idx.size
    dst = np.empty(ns * slot, dtype=np.uint8)
    sizes = (ctypes.c_uint32 * ns)()
    L.jdo_deflate_blocks_mt(sample.ctypes.data, sample.size, BS, 6, dst.ctypes.data, slot,
                            sizes, 16)
    ref = np.frombuffer(sizes, dtype=np.uint32).astype(np.int64)
    assert np.array_equal(ref, csz[idx])
    for j in range(0, ns - 1, 7):        # the oracle's last sample block ends with END
        i = int(idx[j])
        o = int(coff[i])
        got = d_out[o:o + int(csz[i])].cpu().numpy().tobytes()
        assert got == dst[j * slot:j * slot + int(csz[i])].tobytes(), i


@pytest.mark.parametrize("level", [6, 9])
def test_chains_serial_path_is_exact(engine, oracle, monkeypatch, level):
    """k_chains checks that its LDS exchanges were applied in lane order and
    files a block serially otherwise; that path (forced here) gives the same
    chains, so the same output, in block and stream mode"""
    J = engine
    data = J.corpus_mixed(3 * BS + 999, seed=91).tobytes() + bytes(BS)   # incl. a full zero block
    monkeypatch.setenv("JD_CHAINS_SERIAL", "1")
    try:
        g, gs = J.deflate_blocks(data, level=level)
        st = J.deflate_stream(data[:150_000], level=level)
    finally:
        monkeypatch.delenv("JD_CHAINS_SERIAL")
    r, rs = oracle.deflate_blocks(data, level=level)
    assert (g, gs) == (r, rs)
    assert st == oracle.deflate(data[:150_000], level=level)


def test_device_calls_on_two_streams(engine, oracle):
    """the asynchronous entry points share the engine's workspace: a deflate
    on one stream followed at once by a deflate on another must not mix"""
    import torch
    J = engine
    dev = torch.device("cuda", 0)
    outs = []
    datas = [J.corpus_text(8 * BS, seed=s) for s in (1, 2)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    bufs = []
    for data, s in zip(datas, streams):
        n = data.size
        nb = n // BS
        d_in = torch.from_numpy(data).to(dev)
        cap = J.bound(n)
        d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
        d_csz = torch.empty(nb, dtype=torch.int32, device=dev)
        d_coff = torch.empty(nb, dtype=torch.int64, device=dev)
        d_tot = torch.zeros(1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        bufs.append((d_in, d_out, d_csz, d_coff, d_tot))
    for (d_in, d_out, d_csz, d_coff, d_tot), s, data in zip(bufs, streams, datas):
        J.deflate_device(d_in.data_ptr(), data.size, d_out.data_ptr(), d_out.numel(),
                         d_csz.data_ptr(), d_coff.data_ptr(), d_tot.data_ptr(), level=6,
                         stream=s.cuda_stream)
    torch.cuda.synchronize()
    for (d_in, d_out, d_csz, d_coff, d_tot), data in zip(bufs, datas):
        tot = int(d_tot.item())
        r, _ = oracle.deflate_blocks(data.tobytes(), level=6)
        assert d_out[:tot].cpu().numpy().tobytes() == r


@pytest.mark.parametrize("level", [1, 6, 9])
def test_incompressible_blocks_multiphase(engine, oracle, level):
    """Random bytes get near-uniform 8/9-bit literal codes, on which P1's
    lanes never fall into step: P1 gives up on them (flat literal code) and
    k_inflate_mp's multi-phase walks decode them.  Round trip and the
    oracle's inflate of the same stream agree, block by block."""
    import numpy as np
    J = engine
    rng = np.random.default_rng(level)
    data = rng.integers(0, 256, 7 * 65536 + 999, dtype=np.uint8)
    data[3 * 65536:3 * 65536 + 4000] = 7        # one block with a run in it
    comp, sizes = J.deflate_blocks(data.tobytes(), level=level)
    back, us, errs = J.inflate_blocks(comp, sizes)
    assert not any(errs)
    assert back == data.tobytes()
    ref, rus, rer = oracle.inflate_blocks(comp, sizes)
    assert ref == back and list(rus) == list(us)


SLICE_CHILD = r"""
import os, sys, zlib
sys.path.insert(0, os.environ["JD_ROOT"])
import numpy as np
import jdeflate_amd as J
from oracle import jdoracle as O
BS = 65536
rng = np.random.default_rng(5)
data = {"text": J.corpus_text(5 * BS + 4321, seed=21).tobytes(),
        "mixed": J.corpus_mixed(12 * BS, seed=22).tobytes(),
        "zeros": bytes(2 * BS + 5),
        "runs": bytes(np.repeat(rng.choice([0, 1, 255], 3000), rng.integers(1, 120, 3000)).astype(np.uint8))}
for level in (6, 9, 7, 1, 4):
    for name, d in data.items():
        g = J.deflate_blocks(d, level=level)
        r = O.deflate_blocks(d, level=level)
        assert g == r, (name, level)
        assert zlib.decompressobj(-15).decompress(g[0]) == d
print("slices ok")
"""


def test_slice_walk_build_is_bit_exact(engine):
    """The round-6 slice walk (k_chains<4> counting sort + k_match_sl,
    JD_K2_SLICES=1; not the product's default) gives
    the oracle's bytes at every level group, from its own library."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "jdeflate_amd", "lib_sl", "libjdeflate_amd.so")
    if not os.path.exists(lib):
        pytest.skip("slice build not present (build() makes it)")
    env = dict(os.environ, JDAMD_LIB=lib, JD_ROOT=root)
    r = subprocess.run([sys.executable, "-c", SLICE_CHILD], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "slices ok" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])

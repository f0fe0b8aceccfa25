"""The GPU's decomposition of the level 6-9 parser (DESIGN.md "Deflate
pipeline"), modelled on the CPU by tests/support/decomp_emu.c, reproduces
the oracle's tokens and block boundaries exactly.  No GPU."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("emu") / "libemu.so")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so,
                    os.path.join(HERE, "support", "decomp_emu.c")], check=True)
    return ctypes.CDLL(so)


def run_emu(E, d, level):
    tok = np.zeros(max(1, len(d)), np.uint32)
    db = np.zeros(64, np.uint32)
    nt, ndb = ctypes.c_uint32(), ctypes.c_uint32()
    E.emu(d, len(d), level, tok.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nt),
          db.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ndb))
    return [int(x) for x in tok[:nt.value]], [int(x) for x in db[:ndb.value]]


def run_oracle(oracle, d, level):
    t, b, k = [], [], 0
    for x in oracle.trace(d, level=level):
        if x & 0x40000000 and not x & 0x80000000:
            b.append(k)
        else:
            t.append(x)
            k += 1
    return t, b


@pytest.mark.parametrize("level", [6, 7, 8, 9])
def test_decomposition_matches_oracle(emu, oracle, level):
    import jdeflate_amd as J
    try:
        mixed = J.corpus_mixed(12 * 65536, seed=4).tobytes()
        text = J.corpus_text(4 * 65536, seed=3).tobytes()
    except Exception:
        pytest.skip("corpus helper not built")
    rnd = np.random.default_rng(2).integers(0, 256, 65536, dtype=np.uint8).tobytes()
    data = mixed + text + rnd + bytes(65536)
    for b in range(len(data) // 65536):
        d = data[b * 65536:(b + 1) * 65536]
        assert run_emu(emu, d, level) == run_oracle(oracle, d, level), (level, b)


@pytest.mark.parametrize("level", [6, 9])
def test_slice_walk_equals_link_walk(emu, oracle, level):
    """Round 6: the chain of a position as a contiguous slice of the block's
    positions sorted by (bucket, position) -- the representation k_chains<4>
    builds for k_match in block mode -- gives the oracle's tokens too."""
    import jdeflate_amd as J
    try:
        mixed = J.corpus_mixed(8 * 65536, seed=5).tobytes()
        text = J.corpus_text(4 * 65536, seed=6).tobytes()
    except Exception:
        pytest.skip("corpus helper not built")
    data = mixed + text + bytes(65536) + b"ab" * 32768
    flag = ctypes.c_int.in_dll(emu, "emu_slice")
    try:
        flag.value = 1
        for b in range(len(data) // 65536):
            d = data[b * 65536:(b + 1) * 65536]
            assert run_emu(emu, d, level) == run_oracle(oracle, d, level), (level, b)
    finally:
        flag.value = 0

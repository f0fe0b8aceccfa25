"""Buffers that end on a page boundary.

Every device buffer the caller hands over is allocated here with hipMalloc in
whole pages and the data is put flush against the allocation's end, so a read
or write past the caller's last byte touches the next page, which need not be
mapped (torch's caching allocator rounds sizes, so a torch tensor rarely tests
this).  The same tests run on the shipped library (they must be bit-exact
and must not fault) and, in test_bounds_debug_build, in a child process on
the JD_BOUNDS debug build (make EXTRA=-DJD_BOUNDS, jdeflate_amd/lib_dbg),
whose kernels print a JD_BOUNDS line for any access past a buffer's end;
that test fails on any such line.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAGE = 4096
BS = 65536


class _Hip:
    def __init__(self):
        self.L = ctypes.CDLL("libamdhip64.so")
        self.L.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        self.L.hipFree.argtypes = [ctypes.c_void_p]
        self.L.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        self.L.hipDeviceSynchronize.argtypes = []
        self.bufs = []

    def tail(self, n):
        """device address of n bytes that end exactly at a page boundary"""
        size = max(PAGE, -(-n // PAGE) * PAGE)
        p = ctypes.c_void_p()
        assert self.L.hipMalloc(ctypes.byref(p), size) == 0
        self.bufs.append(p.value)
        return p.value + size - n

    def h2d(self, d, a):
        assert self.L.hipMemcpy(d, a.ctypes.data, a.nbytes, 1) == 0

    def d2h(self, a, d):
        # the engine's stream is non-blocking: wait for it first
        assert self.L.hipDeviceSynchronize() == 0
        assert self.L.hipMemcpy(a.ctypes.data, d, a.nbytes, 2) == 0

    def free(self):
        self.L.hipDeviceSynchronize()
        for p in self.bufs:
            self.L.hipFree(p)
        self.bufs = []


def _round_trip(J, data, level):
    """deflate + inflate with every caller buffer flush against a page end"""
    H = _Hip()
    try:
        n = data.size
        nb = max(1, -(-n // BS))
        cap = J.bound(n)
        d_in = H.tail(n)
        H.h2d(d_in, data)
        d_out = H.tail(cap)
        d_csz = H.tail(4 * nb)
        d_coff = H.tail(8 * nb)
        d_tot = H.tail(8)
        J.deflate_device(d_in, n, d_out, cap, d_csz, d_coff, d_tot, level=level)
        tot = np.zeros(1, dtype=np.uint64)
        H.d2h(tot, d_tot)
        total = int(tot[0])
        comp = np.empty(total, dtype=np.uint8)
        csz = np.empty(nb, dtype=np.uint32)
        coff = np.empty(nb, dtype=np.uint64)
        H.d2h(comp, d_out)
        H.d2h(csz, d_csz)
        H.d2h(coff, d_coff)
        # the compressed stream again, now ending at a page end
        d_c = H.tail(total)
        H.h2d(d_c, comp)
        d_cof2 = H.tail(8 * nb)
        H.h2d(d_cof2, coff)
        d_back = H.tail(n)
        d_us = H.tail(4 * nb)
        d_err = H.tail(4 * nb)
        J.inflate_device(d_c, total, d_cof2, d_csz, nb, d_back, d_us, d_err)
        back = np.empty(n, dtype=np.uint8)
        err = np.empty(nb, dtype=np.int32)
        H.d2h(back, d_back)
        H.d2h(err, d_err)
        return comp.tobytes(), csz.tolist(), back, err
    finally:
        H.free()


CASES = [(3 * BS + 1232, "text", 6), (2 * BS - 16, "mixed", 9), (BS + 48, "zero", 6),
         (5 * BS, "text", 1), (4112, "mixed", 6)]


def _data(J, n, kind):
    if kind == "zero":
        return np.zeros(n, dtype=np.uint8)
    return (J.corpus_text if kind == "text" else J.corpus_mixed)(n, seed=n & 0xffff)


@pytest.mark.parametrize("n,kind,level", CASES)
def test_page_end_buffers(engine, oracle, n, kind, level):
    J = engine
    data = _data(J, n, kind)
    comp, sizes, back, err = _round_trip(J, data, level)
    ref, rsizes = oracle.deflate_blocks(data.tobytes(), level=level)
    assert comp == ref and sizes == rsizes
    assert not err.any()
    assert np.array_equal(back, data)


def test_bounds_debug_build(engine):
    """The GPU suite's page-end cases on the JD_BOUNDS build: no access past
    any buffer end (the debug kernels print a JD_BOUNDS line for each)."""
    lib = os.path.join(ROOT, "jdeflate_amd", "lib_dbg", "libjdeflate_amd.so")
    if not os.path.exists(lib):
        pytest.fail("JD_BOUNDS library not built (__graft_entry__.build makes it)")
    code = (
        "import sys; sys.path[:0] = [%r, %r]\n"
        "import numpy as np, jdeflate_amd as J\n"
        "import test_bounds as T\n"
        "for n, kind, level in T.CASES:\n"
        "    d = T._data(J, n, kind)\n"
        "    comp, sizes, back, err = T._round_trip(J, d, level)\n"
        "    assert not err.any() and np.array_equal(back, d), (n, kind)\n"
        "    out, r, e = J.Inflator().decompress(comp + bytes(8), chunk=5000, tgt=70000, final='never')\n"
        "    assert out == d.tobytes(), (n, kind, r, e)\n"
        "print('done')\n" % (ROOT, os.path.join(ROOT, "tests")))
    env = dict(os.environ, JDAMD_LIB=lib)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                       timeout=240, cwd=ROOT)
    out = p.stdout + p.stderr
    assert p.returncode == 0 and "done" in p.stdout, out[-3000:]
    bad = [l for l in out.splitlines() if "JD_BOUNDS" in l]
    assert not bad, "\n".join(bad[:20])


def test_bad_links_never_fault(engine):
    """Hash-4 links longer than their position (the JD_TEST_BADLINKS hook
    replaces about half of them) must never make a walk read outside the
    chains or the input (held_long's `q = cur - d` wrapped
    and the window test still passed).  On the JD_BOUNDS build: no fault, no
    JD_BOUNDS line, and the output is still a valid encoding of the input
    (every match is checked against the bytes), in block and stream mode."""
    lib = os.path.join(ROOT, "jdeflate_amd", "lib_dbg", "libjdeflate_amd.so")
    if not os.path.exists(lib):
        pytest.fail("JD_BOUNDS library not built (__graft_entry__.build makes it)")
    code = (
        "import sys, zlib; sys.path[:0] = [%r]\n"
        "import jdeflate_amd as J\n"
        "n = 0\n"
        "for size, kind, level in [(4 << 20, 'text', 6), (2 << 20, 'text', 7), (1 << 20, 'mixed', 9)]:\n"
        "    d = (J.corpus_text if kind == 'text' else J.corpus_mixed)(size, seed=5).tobytes()\n"
        "    out, sizes = J.deflate_blocks(d, level=level)\n"
        "    assert zlib.decompress(out, -15) == d, (kind, level)\n"
        "    n += 1\n"
        "for level in (6, 9):\n"
        "    d = J.corpus_text(60000, seed=9).tobytes()\n"
        "    out = J.deflate_stream(d, level=level)\n"
        "    assert zlib.decompress(out, -15) == d, level\n"
        "    n += 1\n"
        "print('done', n)\n" % ROOT)
    env = dict(os.environ, JDAMD_LIB=lib, JD_TEST_BADLINKS="1")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                       timeout=240, cwd=ROOT)
    out = p.stdout + p.stderr
    assert p.returncode == 0 and "done 5" in p.stdout, out[-3000:]
    bad = [l for l in out.splitlines() if "JD_BOUNDS" in l]
    assert not bad, "\n".join(bad[:20])

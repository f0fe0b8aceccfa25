"""dev: per-block k_pjoin statistics (debug build with -DJD_PJSTATS)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["JD_PARSE"] = "split"
import jdeflate_amd as J
L = J.load_library(os.path.join(ROOT, "jdeflate_amd", "lib_dbg", "libjdeflate_amd.so"))
BS = 65536
for name, data, lvl in (("text", J.corpus_text(16 * BS, seed=5), 6),
                        ("mixed", J.corpus_mixed(48 * BS, seed=9), 9),
                        ("mixed", J.corpus_mixed(48 * BS, seed=9), 6)):
    d = data.tobytes()
    nb = len(d) // BS
    tok = np.zeros(nb * BS, np.uint32)
    dbi = np.zeros(nb * 65, np.uint32)
    r = L.jdgpu_debug_deflate(d, len(d), BS, lvl, tok.ctypes.data, dbi.ctypes.data, None)
    assert r == 0, r
    dbi = dbi.reshape(nb, 65)
    print(f"== {name} L{lvl}: serial d1 end batch ev rejoin dg ds | low% ndb")
    tot = np.zeros(6, np.int64)
    for b in range(nb):
        blk = np.frombuffer(d[b * BS:(b + 1) * BS], np.uint8)
        low = (blk < 16).mean() * 100
        q = dbi[b, 57:65]
        tot += q[:6]
        print(f"  {b:3d}: {' '.join(f'{int(v):6d}' for v in q)} | {low:5.1f} {int(dbi[b,0])}")
    print("  total", tot)

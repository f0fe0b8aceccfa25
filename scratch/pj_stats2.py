"""dev: worst blocks of k_pjoin over a large mixed sample (debug build)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["JD_PARSE"] = "split"
import jdeflate_amd as J
L = J.load_library(os.path.join(ROOT, "jdeflate_amd", "lib_dbg", "libjdeflate_amd.so"))
BS = 65536
nb = 4096
for lvl in (9, 6):
    data = J.corpus_mixed(nb * BS, seed=1)
    d = data.tobytes()
    tok = np.zeros(nb * BS, np.uint32)
    dbi = np.zeros(nb * 65, np.uint32)
    r = L.jdgpu_debug_deflate(d, len(d), BS, lvl, tok.ctypes.data, dbi.ctypes.data, None)
    assert r == 0, r
    q = dbi.reshape(nb, 65)[:, 57:65].astype(np.int64)
    blk = np.frombuffer(d, np.uint8).reshape(nb, BS)
    low = (blk < 16).mean(axis=1) * 100
    print(f"L{lvl} totals serial d1 end batch ev rejoin:", q[:, :6].sum(0), flush=True)
    for b in np.argsort(-q[:, 0])[:12]:
        print(f"  blk {b:5d} serial {q[b,0]:6d} d1 {q[b,1]:5d} end {q[b,2]:3d} batch {q[b,3]:5d} ev {q[b,4]:4d} rejoin {q[b,5]:5d} mask {q[b,6]} ds {q[b,7]} low {low[b]:5.1f}", flush=True)

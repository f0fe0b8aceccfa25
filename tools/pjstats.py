"""k_pjoin step statistics (build with -DJD_PJSTATS): serial steps, d1 stops,
list ends, batches, events, rejoins per 64 KiB block"""
import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import jdeflate_amd as J
from jdeflate_amd import engine as E
L = E.load_library()
n = 64 << 20
for name, data in (("text", J.corpus_text(n, seed=1000, threads=16)), ("mixed", J.corpus_mixed(n, seed=1000, threads=16))):
    nb = n // 65536
    tok = np.empty(n, dtype=np.uint32)
    dbi = np.zeros(nb * 65, dtype=np.uint32)
    rec = np.empty(n, dtype=np.uint64)
    r = L.jdgpu_debug_deflate(data.ctypes.data_as(ctypes.c_char_p), n, 65536, 6,
                              tok.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                              dbi.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                              rec.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    q = dbi.reshape(nb, 65)[:, 65 - 8:]
    print(name, r, "per block: serial %.0f d1 %.1f end %.1f batch %.0f ev %.1f rejoin %.1f" % tuple(q[:, :6].mean(0)), flush=True)

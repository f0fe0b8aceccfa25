import os, sys, numpy as np
os.environ["JD_NOFALLBACK"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jdeflate_amd as J
from oracle import jdoracle as O
n = 1 << 30
for name, gen in (("text", J.corpus_text), ("mixed", J.corpus_mixed)):
    data = gen(n, seed=1000, threads=16)
    g, gs = J.deflate_blocks(data.tobytes(), level=6)
    try:
        back, us, er = J.inflate_blocks(g, gs)
    except Exception as ex:
        print("exc", ex)
    import ctypes
    L = J.load_library()
    nb = len(gs)
    usz = (ctypes.c_uint32 * nb)(); err = (ctypes.c_int32 * nb)()
    dst = ctypes.create_string_buffer(nb * 65536)
    L.jdgpu_inflate(g, len(g), (ctypes.c_uint32 * nb)(*gs), nb, 65536, dst, usz, err)
    fb = [(i, usz[i]) for i in range(nb) if usz[i] >= 0xF0000000]
    print(name, "fallback blocks", len(fb), [(i, hex(u)) for i, u in fb[:8]])
    offs = np.concatenate([[0], np.cumsum(gs)])
    for i, u in fb[:3]:
        t = O.trace(data[i*65536:(i+1)*65536].tobytes(), level=6)
        nm = sum(1 for x in t if x & 0x80000000)
        print("  block", i, "matches", nm, "tokens", len(t))

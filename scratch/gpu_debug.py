import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import jdeflate_amd as J
from jdeflate_amd import engine as E
from oracle import jdoracle as O
L = E.load_library()
L.jdgpu_debug_deflate.restype = ctypes.c_int
L.jdgpu_debug_deflate.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
m = J.corpus_mixed(16 * 65536, seed=4).tobytes()
for lvl, blk in ((6, 0), (7, 11)):
    d = m[blk * 65536:(blk + 1) * 65536]
    tok = np.zeros(65536, np.uint32); dbi = np.zeros(65, np.uint32); rec = np.zeros(65536, np.uint64)
    r = L.jdgpu_debug_deflate(d, len(d), 65536, lvl, tok.ctypes.data, dbi.ctypes.data, rec.ctypes.data)
    ntok = int(dbi[2 * int(dbi[0]) - 1])
    gt = [int(x) for x in tok[:ntok]]
    ot = O.trace(d, level=lvl)
    ob = [x for x in ot if x & 0x40000000 and not x & 0x80000000]
    ot2 = [x for x in ot if not (x & 0x40000000 and not x & 0x80000000)]
    print(f"L{lvl} blk{blk}: ndb={dbi[0]} gpu tokens {len(gt)} oracle tokens {len(ot2)} oracle blocks {len(ob)}")
    print(" gpu db:", [(int(dbi[1+2*i]), int(dbi[2+2*i])) for i in range(int(dbi[0]))])
    # oracle block boundaries in token index
    k = 0; bounds = []
    for x in ot:
        if x & 0x40000000 and not x & 0x80000000: bounds.append(k)
        else: k += 1
    print(" ora db ends:", bounds)
    # decode to (pos, tok) and find first diff
    pos = 0
    for i, (a, b) in enumerate(zip(gt, ot2)):
        if a != b:
            def f(t): return ("M", (t >> 16) & 0x7fff, t & 0xffff) if t & 0x80000000 else ("L", t)
            print(f" first diff at token {i} pos {pos}: gpu {f(a)} ora {f(b)}")
            for q in range(max(0, pos - 3), pos + 4):
                rr = int(rec[q]); print(f"   rec[{q}] l48={rr & 511} o48={(rr >> 9) & 0x7fff} l24={(rr >> 24) & 511} o24={(rr >> 33) & 0x7fff} s3={rr >> 48}")
            print("   bytes", d[max(0,pos-8):pos+16])
            print("   prev tokens gpu", [f(x) for x in gt[max(0,i-5):i+3]])
            print("   prev tokens ora", [f(x) for x in ot2[max(0,i-5):i+3]])
            break
        pos += ((a >> 16) & 0x7fff) if a & 0x80000000 else 1
    else:
        print(" tokens identical for common prefix")

import sys, os, ctypes
sys.path.insert(0, '/root/repo')
import numpy as np
import jdeflate_amd as J
from oracle import jdoracle as O
E = ctypes.CDLL('scratch/libemu.so')
def emu(d, lvl):
    tok = np.zeros(65536, np.uint32); nt = ctypes.c_uint32(); db = np.zeros(64, np.uint32); ndb = ctypes.c_uint32()
    E.emu(d, len(d), lvl, tok.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nt), db.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ndb))
    return [int(x) for x in tok[:nt.value]], [int(x) for x in db[:ndb.value]]
def ora(d, lvl):
    ot = O.trace(d, level=lvl); k = 0; b = []; t = []
    for x in ot:
        if x & 0x40000000 and not x & 0x80000000: b.append(k)
        else: t.append(x); k += 1
    return t, b
m = J.corpus_mixed(16 * 65536, seed=4).tobytes()
t = J.corpus_text(8 * 65536, seed=3).tobytes()
for lvl in (6, 7, 8, 9):
    for name, data in (("mixed", m), ("text", t)):
        for blk in range(len(data) // 65536):
            d = data[blk * 65536:(blk + 1) * 65536]
            a, ab = emu(d, lvl); o, obd = ora(d, lvl)
            if a != o or ab != obd:
                i = next((i for i, (x, y) in enumerate(zip(a, o)) if x != y), None)
                print(f"L{lvl} {name} blk{blk}: MISMATCH ntok {len(a)} vs {len(o)} dbs {ab} vs {obd} first diff tok {i}")
print("done")

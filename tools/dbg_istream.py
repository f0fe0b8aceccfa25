"""debug: IStream with tiny targets on a zlib stream"""
import os, sys, zlib, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jdeflate_amd import engine as E
import jdeflate_amd as J
data = J.corpus_text(3000, seed=11).tobytes()
c = zlib.compressobj(6, zlib.DEFLATED, -15)
comp = c.compress(data) + c.flush()
buf = ctypes.create_string_buffer(comp, len(comp))
base = ctypes.addressof(buf)
s = E.IStream()
out = b""
pos = 0
for k in range(8):
    st, err, prod, cons, _ = s.inflate(len(comp) - pos, 1, src_addr=base + pos)
    out += s.out.raw[:prod]
    pos += cons
    print("cached", k, st, err, prod, cons, pos, out, data[:len(out)] == out, flush=True)
    if st != E.IS_FULL:
        break
inf = E.Inflator()
out, r, err = inf.decompress(comp, chunk=20000, tgt=1, final="never")
print("inflator", r, err, out[:20], out == data)

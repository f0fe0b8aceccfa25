import os, sys, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jdeflate_amd as J
from oracle import jdoracle as O
BS = 65536
n = int(os.environ.get("SIZE", str(1 << 30)))
data = J.corpus_text(n, seed=1000, threads=16)
g, gs = J.deflate_blocks(data.tobytes(), level=6)
back, us, er = J.inflate_blocks(g, gs)
bad = [i for i, e in enumerate(er) if e]
print("nblocks", len(gs), "bad", len(bad), "first", bad[:10], "codes", sorted(set(er[i] for i in bad)))
offs = np.concatenate([[0], np.cumsum(gs)])
for i in bad[:3]:
    blk = g[offs[i]:offs[i + 1]]
    o, u, e = J.inflate_blocks(blk, [gs[i]])
    ro, ru, re_ = O.inflate_blocks(blk, [gs[i]])
    print("block", i, "alone: err", e, "usize", u, "oracle", re_, ru, "match", o == ro)
# position dependence: the same blocks at various chunk positions
for k in (64, 256, 1024, 4096):
    if k > len(gs): break
    sub = g[:offs[k]]
    o, u, e = J.inflate_blocks(sub, gs[:k])
    print("first", k, "blocks: bad", sum(1 for x in e if x))

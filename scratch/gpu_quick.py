"""Quick GPU parity probe (dev only)."""
import sys, time, zlib, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import jdeflate_amd as J
from oracle import jdoracle as O
print("available", J.available(), flush=True)
cases = []
t = J.corpus_text(8 * 65536 + 777, seed=3).tobytes()
m = J.corpus_mixed(16 * 65536, seed=4).tobytes()
rnd = np.random.default_rng(5).integers(0, 256, 3 * 65536, dtype=np.uint8).tobytes()
cases = [("text", t), ("mixed", m), ("rand", rnd), ("empty", b""), ("one", b"a"), ("zeros", bytes(200000)),
         ("abc", b"ABCDEFGHIJABCDEFGHIJ"), ("small", t[:1000])]
bad = 0
for lvl in (6, 9, 7, 8, 1, 3, 5, 0):
    for name, d in cases:
        try:
            g, gs = J.deflate_blocks(d, level=lvl)
        except Exception as e:
            print("EXC", lvl, name, e, flush=True); bad += 1; continue
        r, rs = O.deflate_blocks(d, level=lvl)
        ok = g == r and gs == rs
        if not ok:
            bad += 1
            # find first differing block
            off = 0
            for i, (a, b) in enumerate(zip(gs, rs)):
                if a != b or g[off:off+a] != r[off:off+b]:
                    gb, rb = g[off:off+a], r[off:off+b]
                    k = next((j for j in range(min(len(gb), len(rb))) if gb[j] != rb[j]), min(len(gb), len(rb)))
                    print(f"  block {i}: gpu {a} ref {b} first diff byte {k}", flush=True)
                    break
                off += a
        back, us, er = J.inflate_blocks(g, gs)
        iok = back == d and not any(er)
        zok = zlib.decompressobj(-15).decompress(g) == d
        print(f"L{lvl} {name:6s} n={len(d):7d} gpu={len(g):7d} ref={len(r):7d} deflate_parity={ok} inflate_ok={iok} zlib={zok} errs={set(er)}", flush=True)
        bad += (not iok) + (not zok)
# single-stream inflate via the drop-in API on a zlib stream
d = t[:300000]
c = zlib.compressobj(9, zlib.DEFLATED, -15); zc = c.compress(d) + c.flush()
inf = J.Inflator(); out, rr, ee = inf.decompress(zc, chunk=10000, tgt=65536)
print("inflator drop-in zlib stream:", out == d, rr, ee)
dfl = J.Deflator(6); cc = dfl.compress(d, chunk=50000, tgt=30000)
print("deflator drop-in:", cc == O.deflate_blocks(d)[0], zlib.decompressobj(-15).decompress(cc) == d)
# throughput probe (host API, includes copies)
big = J.corpus_text(256 << 20, seed=1).tobytes()
J.deflate_blocks(big[:1 << 20])
t0 = time.time(); g, gs = J.deflate_blocks(big); t1 = time.time()
back, us, er = J.inflate_blocks(g, gs); t2 = time.time()
print(f"256MiB host-API deflate {256/(t1-t0):.1f} MB/s inflate {256/(t2-t1):.1f} MB/s ratio {len(g)/len(big):.4f} ok={back==big}")
print("BAD", bad)

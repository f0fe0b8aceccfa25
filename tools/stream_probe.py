"""Stream-mode parity probe: GPU single-window deflate vs the oracle; prints
the first mismatching case with the first differing byte."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import jdeflate_amd as J
from oracle import jdoracle as O
C1 = b"The quick brown fox jumps over the lazy dog. "
text = J.corpus_text(3 << 20, seed=31).tobytes()
mixed = J.corpus_mixed(2 << 20, seed=32).tobytes()
rng = np.random.default_rng(5)
cases = [("empty", b""), ("one", b"x"), ("short", text[:100]), ("64k", text[:65536]),
         ("128k", text[:131072]), ("200k", text[:200000]), ("c1", (C1 * 30000)[:1 << 20]),
         ("text1m", text[:1 << 20]), ("text3m", text), ("mixed2m", mixed),
         ("random", rng.integers(0, 256, 300000, dtype=np.uint8).tobytes()), ("zeros", bytes(300000))]
for k in range(-300, 700, 97):
    cases.append((f"t{131072 + k}", text[:131072 + k]))
    cases.append((f"m{131072 + 98304 + k}", mixed[:131072 + 98304 + k]))
    cases.append((f"g{65536 + k}", text[:65536 + k]))
bad = 0
for level in (6, 9, 0, 7, 8, 1, 2, 3, 4, 5):
    for name, d in cases:
        t0 = time.time()
        try:
            g = J.deflate_stream(d, level=level)
        except Exception as e:
            print("EXC", level, name, e, flush=True); bad += 1; continue
        t1 = time.time()
        r = O.deflate(d, level=level)
        if g != r:
            bad += 1
            k = next((i for i in range(min(len(g), len(r))) if g[i] != r[i]), min(len(g), len(r)))
            print(f"MISMATCH L{level} {name} n={len(d)} gpu={len(g)} ref={len(r)} firstdiff={k}", flush=True)
        else:
            print(f"ok L{level} {name} n={len(d)} out={len(g)} gpu_ms={1e3*(t1-t0):.1f}", flush=True)
print("BAD", bad)

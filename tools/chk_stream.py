import os, sys
sys.path.insert(0, os.getcwd())
import jdeflate_amd as J
from oracle import jdoracle as O
mixed = J.corpus_mixed(2 << 20, seed=32).tobytes()
for n in (150_000, 300_000, 600_000, 1 << 20, 2 << 20):
    for lv in (1, 6):
        for ser in ("0", "1"):
            os.environ["JD_CHAINS_SERIAL"] = ser
            g = J.deflate_stream(mixed[:n], level=lv)
            r = O.deflate(mixed[:n], level=lv)
            d = next((i for i in range(min(len(g), len(r))) if g[i] != r[i]), None)
            print(n, lv, ser, len(g), len(r), g == r, d, flush=True)

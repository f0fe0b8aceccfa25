import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import jdeflate_amd as J
from jdeflate_amd import engine as E
from oracle import jdoracle as O
import tokens as T
for n, seed in ((700000, 41), (700000, 7), (1 << 20, 41), (400000, 41)):
    data = J.corpus_text(n, seed=seed).tobytes()
    want = O.deflate(data, 6)
    a = T.tokens(want)
    for rep in range(3):
        got = E.deflate_stream(data, 6)
        if got == want:
            print(n, seed, rep, "ok", flush=True); continue
        b = T.tokens(got); pos = 0
        for i, (x, y) in enumerate(zip(a, b)):
            if x != y:
                print(n, seed, rep, "diff pos", pos, "want", x, "got", y, flush=True); break
            if x[0] == "L": pos += 1
            elif x[0] == "M": pos += x[1]

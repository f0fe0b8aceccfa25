"""debug: pieces of a single-window stream through jdgpu_stream_*, return codes"""
import ctypes, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jdeflate_amd as J
from jdeflate_amd import engine as E
from oracle import jdoracle as O
L = E.load_library()
level = int(os.environ.get("LEVEL", "6"))
data = J.corpus_text(700_000, seed=41).tobytes()
s = L.jdgpu_stream_create(level, 0, None, 0)
prev = 0
outs = []
for end in list(range(100_000, len(data), 100_000)) + [len(data)]:
    fl = 1 if end == len(data) else 2
    piece = data[prev:end]
    cap = int(L.jdgpu_stream_bound(len(piece))) + 64
    out = ctypes.create_string_buffer(cap)
    ce = (ctypes.c_uint64 * 1)(len(piece))
    r = L.jdgpu_stream_deflate(s, piece, len(piece), ce, 1, fl, out, cap)
    print("piece", prev, end, "->", r, flush=True)
    if r < 0:
        break
    outs.append(out.raw[:r])
    prev = end
L.jdgpu_stream_destroy(s)
got = b"".join(outs)
want = O.deflate_calls(data, [(e, 2) for e in range(100_000, len(data), 100_000)] + [(len(data), 1)], level)
print("equal", got == want, len(got), len(want))
if got != want:
    i = next(i for i in range(min(len(got), len(want))) if got[i] != want[i])
    print("first diff at", i)

"""Single-window (DEFLT_SINGLEWINDOW) deflate rate and its per-kernel times:
SIZE bytes of the bench text (default 64 MiB), level LEVEL, one call through
jdgpu_deflate_stream (host buffers: PCIe included), then the output checked
by zlib.  Prints one JSON line."""
import json
import os
import sys
import time
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jdeflate_amd as J

n = int(os.environ.get("SIZE", str(64 << 20)))
level = int(os.environ.get("LEVEL", "6"))
data = J.corpus_text(n, seed=1000, threads=16).tobytes()
J.deflate_stream(data[:1 << 20], level=level)          # warm-up
J.prof_enable(True)
t0 = time.perf_counter()
out = J.deflate_stream(data, level=level)
el = time.perf_counter() - t0
kt = J.prof_read()
J.prof_enable(False)
ok = zlib.decompressobj(-15).decompress(out) == data
print(json.dumps({"bytes": n, "level": level, "out": len(out), "ok": ok, "s": round(el, 3),
                  "MBps": round(n / el / 1e6, 1),
                  **{k: round(v[0], 2) for k, v in kt.items() if v[0] > 0.05}}), flush=True)

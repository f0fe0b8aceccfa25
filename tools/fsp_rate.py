"""Decode rate of zlib-made streams (no sync markers) through jdgpu_istream,
one call with the whole input, parallel rounds on and off; per-kernel times."""
import ctypes, json, os, sys, time, zlib
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jdeflate_amd as J
from jdeflate_amd import engine as E

n = int(os.environ.get("SIZE", str(256 << 20)))
lvl = int(os.environ.get("LEVEL", "6"))
data = J.corpus_text(n, seed=77, threads=16).tobytes()
t = time.time()
c = zlib.compressobj(lvl, zlib.DEFLATED, -15)
comp = c.compress(data) + c.flush()
print(f"zlib L{lvl}: {n} -> {len(comp)} in {time.time() - t:.1f}s", flush=True)
src = ctypes.create_string_buffer(comp, len(comp))
out = ctypes.create_string_buffer(n + 1)


def run(fsp, m=None):
    s = E.IStream()
    s.fsp(fsp)
    sub = comp if m is None else comp[:m]
    buf = src if m is None else ctypes.create_string_buffer(sub, len(sub))
    t = time.time()
    st, err, prod, used, par = s.inflate(len(sub), n + 1, src_addr=ctypes.addressof(buf), out=out)
    dt = time.time() - t
    r = s.fsp()
    s.close()
    return st, prod, dt, r


run(1)     # warm
J.prof_enable(True)
st, prod, dt, r = run(1)
prof = J.prof_read()
J.prof_enable(False)
ok = st == E.IS_ENDED and out.raw[:prod] == data
print(json.dumps({"fsp": 1, "status": st, "ok": ok, "bytes": prod, "s": round(dt, 4),
                  "MB_s": round(prod / dt / 1e6, 1), "rounds": r[0], "chunks": r[1],
                  "kernels_ms": {k: round(v[0], 3) for k, v in prof.items()},
                  "launches": {k: v[1] for k, v in prof.items()}}), flush=True)
m = len(comp) // 16
st, prod, dt, r = run(0, m)
print(json.dumps({"fsp": 0, "sample_in": m, "bytes": prod, "s": round(dt, 4),
                  "MB_s": round(prod / dt / 1e6, 1)}), flush=True)

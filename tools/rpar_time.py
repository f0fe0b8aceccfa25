"""Phase times of the parallel resume (k_inflate_rpar) on the drop-in stream
pattern (32 KiB reads, 64 KiB targets): one JD_IS_TRACE line per launch with
its decode and LDS-resolve microseconds, then their means."""
import os, re, subprocess, sys
if os.environ.get("JD_IS_TRACE") != "1":
  for aw, nw in (("0", "4"), ("1", "4"), ("1", "8")):
    env = dict(os.environ, JD_IS_TRACE="1", JD_RPALLW=aw, JD_RPNW=nw)
    r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True, text=True)
    lines = [l for l in r.stderr.splitlines() if l.startswith("IST rpar")]
    print(f"JD_RPALLW={aw} JD_RPNW={nw}")
    for l in lines[:6]:
        print(l)
    dec = [float(m.group(1)) for l in lines for m in [re.search(r"decode_us=([\d.]+)", l)] if m]
    res = [float(m.group(1)) for l in lines for m in [re.search(r"resolve_us=([\d.]+)", l)] if m]
    prod = [int(m.group(1)) for l in lines for m in [re.search(r"prod=(\d+)", l)] if m]
    recs = [int(m.group(1)) for l in lines for m in [re.search(r"recs=(\d+)", l)] if m]
    ph = {k: [float(m.group(1)) for l in lines for m in [re.search(k + r"_us=([\d.]+)", l)] if m]
          for k in ("hdr", "walk", "chain", "write")}
    n = max(len(dec), 1)
    print("  phases (mean us): " + ", ".join(f"{k} {sum(v) / n:.1f}" for k, v in ph.items()))
    print(f"launches {len(dec)}: mean decode {sum(dec) / n:.1f} us, mean resolve {sum(res) / n:.1f} us, "
          f"mean output {sum(prod) / n:.0f} B, mean records {sum(recs) / n:.0f}; rc {r.returncode}", flush=True)
    if r.returncode:
        print(r.stderr[-2000:])
        sys.exit(r.returncode)
  sys.exit(0)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jdeflate_amd as J
from jdeflate_amd import engine as E
text = J.corpus_text(4 << 20, seed=7).tobytes()
comp = J.deflate_blocks(text, level=6)[0]
s = E.IStream()
out, pos = bytearray(), 0
while True:
    st, err, prod, cons, _ = s.inflate(comp[pos:pos + 32768], 65536)
    out += s.out.raw[:prod]
    pos += cons
    if st == E.IS_FULL:
        continue
    if st != E.IS_NEEDINPUT or pos >= len(comp):
        break
s.close()
assert bytes(out) == text

"""Phase clocks of the parallel resume (k_inflate_rpar) behind the drop-in
inflator: a build with -DRP_CLOCK prints one line per launch (tools/var/<name>,
see tools/variants.sh); this drives the stream decoder with 32 KiB reads and
64 KiB targets on SIZE bytes of text (this library's blocks, then zlib's
stream) and prints the mean phase times per launch in microseconds.

    JDAMD_LIB=tools/var/rpclock/libjdeflate_amd.so python tools/rpar_clock.py
"""
import json
import os
import re
import subprocess
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(kind: str) -> None:
    sys.path.insert(0, ROOT)
    import jdeflate_amd as J
    from jdeflate_amd import engine as E
    n = int(os.environ.get("SIZE", str(4 << 20)))
    text = J.corpus_text(n, seed=1000).tobytes()
    if kind == "blocks":
        comp = J.deflate_blocks(text, level=6)[0]
    else:
        c = zlib.compressobj(6, zlib.DEFLATED, -15, 9)
        comp = c.compress(text) + c.flush()
    s = E.IStream()
    out, off, calls = [], 0, 0
    t0 = time.perf_counter()
    while off < len(comp):
        piece = comp[off:off + 32768]
        done = 0
        while True:
            st, err, prod, cons, _ = s.inflate(piece[done:], 65536)
            out.append(s.out.raw[:prod])
            done += cons
            calls += 1
            if st != E.IS_FULL:
                break
        off += len(piece)
        if st in (E.IS_ENDED, E.IS_ERROR):
            break
    el = time.perf_counter() - t0
    ok = b"".join(out) == text
    print(json.dumps({"kind": kind, "ok": ok, "calls": calls, "MBps": round(n / el / 1e6, 1),
                      "us_per_call": round(el / calls * 1e6, 1)}), flush=True)


def main() -> None:
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    for kind in ("blocks", "zlib"):
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", kind],
                           capture_output=True, text=True, timeout=600)
        lines = r.stdout.splitlines()
        rows = [l for l in lines if l.startswith("RPC ")]
        tail = [l for l in lines if l.startswith("{")]
        keys = ["in", "out", "rec", "hdr", "a1", "a2", "chain", "write", "rest", "resolve", "copy"]
        acc = {k: 0.0 for k in keys}
        for l in rows:
            for k, v in re.findall(r"(\w+)=([\d.]+)", l):
                if k in acc:
                    acc[k] += float(v)
        m = len(rows) or 1
        print(kind, tail[-1] if tail else r.stderr[-2000:], flush=True)
        print(f"  launches {len(rows)}: " + " ".join(f"{k}={acc[k] / m:.1f}" for k in keys), flush=True)


if __name__ == "__main__":
    main()

"""Per-kernel regression gate: fail when any kernel got more than 5 % slower.

    python tools/kernel_regress.py NEW BASE [--tol 0.05] [--min-ms 0.1]

NEW and BASE are each one of
  * a rocprofv3 `--stats` CSV (profiles/rXX_*_kernel_stats.csv): AverageNs per launch;
  * a bench.py JSON line (or a file holding one, e.g. BENCH_rXX.json's "parsed"):
    config.kernel_ms_per_step;
  * a tools/ab_probe.py JSON line: per-kernel ms per launch.
Kernel names are normalised so that template arguments that only select a
variant (k_chains<3, false, 1> vs k_chains<3, false>, k_match<false>) compare
equal: the name before '(' without 'void ', keeping only a leading numeric
template argument.  Only this engine's kernels (k_*) are compared; kernels
under --min-ms in BASE are not gated (launch noise).  Exit status 1 lists
every kernel over the tolerance.
"""
import argparse
import csv
import json
import re
import sys


def norm(name: str) -> str:
    s = name.strip().strip('"')
    s = s.split("(")[0]
    if s.startswith("void "):
        s = s[5:]
    m = re.match(r"^([A-Za-z_]\w*)(?:<\s*([^,>]*)[^>]*>)?$", s)
    if not m:
        return s
    base, first = m.group(1), m.group(2)
    return f"{base}<{first.strip()}>" if first and first.strip().isdigit() else base


def load(path: str) -> dict:
    txt = open(path).read()
    if txt.lstrip().startswith('"Name"') or txt.lstrip().startswith("Name"):
        out = {}
        for row in csv.DictReader(txt.splitlines()):
            out[norm(row["Name"])] = float(row["AverageNs"]) / 1e6
        return out
    for line in txt.splitlines()[::-1]:
        line = line.strip()
        if not line.startswith("{"):
            continue
        d = json.loads(line) if line.endswith("}") else None
        if d is None:
            continue
        if "parsed" in d:
            d = d["parsed"]
        if "config" in d and "kernel_ms_per_step" in d["config"]:
            return {norm(k): v for k, v in d["config"]["kernel_ms_per_step"].items()}
        return {norm(k): v for k, v in d.items() if isinstance(v, (int, float)) and k.startswith("k_")}
    d = json.loads(txt)
    if "parsed" in d:
        d = d["parsed"]
    return {norm(k): v for k, v in d["config"]["kernel_ms_per_step"].items()}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("new")
    ap.add_argument("base")
    ap.add_argument("--tol", type=float, default=0.05)
    ap.add_argument("--min-ms", type=float, default=0.5)
    a = ap.parse_args()
    new, base = ({k: v for k, v in load(p).items() if k.startswith("k_")} for p in (a.new, a.base))
    bad = []
    for k in sorted(base, key=lambda k: -base[k]):
        b = base[k]
        if b < a.min_ms or k not in new:
            continue
        r = new[k] / b - 1
        flag = "SLOWER" if r > a.tol else ""
        print(f"{k:24s} {b:9.3f} -> {new[k]:9.3f} ms  {r * 100:+6.1f} % {flag}")
        if flag:
            bad.append(k)
    for k in sorted(set(new) - set(base)):
        if new[k] >= a.min_ms:
            print(f"{k:24s}       new -> {new[k]:9.3f} ms")
    if bad:
        print(f"FAIL: {len(bad)} kernel(s) more than {a.tol * 100:.0f} % slower: {', '.join(bad)}")
        return 1
    print("ok: no kernel more than %.0f %% slower" % (a.tol * 100))
    return 0


if __name__ == "__main__":
    sys.exit(main())

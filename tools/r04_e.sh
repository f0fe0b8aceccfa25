#!/bin/bash
# k_inflate_par batch cadence / store-cost probes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s5
mkdir -p $O
cd $R
bash tools/variants.sh run base p1k8 p1k2 p1ns p1k8r16 p1wc base p1wc > $O/var.log 2>&1 || { tail -5 $O/var.log; exit 3; }
python3 - $O/var.log <<'PY'
import sys, json
n=None
for l in open(sys.argv[1]):
    if l.startswith("=="): n=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(n, d["wall_ms"], d["ok"], "par", d["k_inflate_par"], "res", d["k_inflate_resolve"], "mp", d.get("k_inflate_mp"), "inflate", d.get("k_inflate"))
PY

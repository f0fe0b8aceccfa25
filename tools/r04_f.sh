#!/bin/bash
# k_chains: batch loop without byte-wise global loads (prefetch stays in flight)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s6
mkdir -p $O
cd $R
bash tools/variants.sh run ch chd ch chd > $O/var.log 2>&1 || { tail -5 $O/var.log; exit 3; }
python3 - $O/var.log <<'PY'
import sys, json
n=None
for l in open(sys.argv[1]):
    if l.startswith("=="): n=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(n, d["wall_ms"], d["ok"], d["outcrc"], "c4", d["k_chains<4>"], "c3", d["k_chains<3>"], "match", d["k_match"])
PY

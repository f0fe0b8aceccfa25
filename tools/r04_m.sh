#!/bin/bash
# k_chains: filing split over CH_FW waves by bucket residue
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s14
mkdir -p $O
cd $R
bash tools/variants.sh run fw1 fw2 fw4 fw1 fw4 > $O/var.log 2>&1 || { tail -5 $O/var.log; exit 3; }
python3 - $O/var.log <<'PY'
import sys, json
n=None
for l in open(sys.argv[1]):
    if l.startswith("=="): n=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(n, d["wall_ms"], d["ok"], d["outcrc"], "c4", d["k_chains<4>"], "c3", d["k_chains<3>"])
PY

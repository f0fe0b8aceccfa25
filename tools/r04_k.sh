#!/bin/bash
# k_inflate_resolve: copy loads issued in batches of RS_B steps
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s15
mkdir -p $O
cd $R
bash tools/variants.sh run rs8 rs6 rs5 rs8 rs6 rs5 > $O/var.log 2>&1 || { tail -5 $O/var.log; exit 3; }
python3 - $O/var.log <<'PY'
import sys, json
n=None
for l in open(sys.argv[1]):
    if l.startswith("=="): n=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(n, d["wall_ms"], d["ok"], "res", d["k_inflate_resolve"], "par", d["k_inflate_par"])
PY

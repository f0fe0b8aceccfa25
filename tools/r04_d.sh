#!/bin/bash
# k_match: links chased ahead of the quick rejects (K2_SPEC) A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4
mkdir -p $O
cd $R
bash tools/variants.sh run base spec4 spec6 spec3 base spec4 > $O/var.log 2>&1 || { tail -5 $O/var.log; exit 3; }
python3 - $O/var.log <<'PY'
import sys, json
n=None
for l in open(sys.argv[1]):
    if l.startswith("=="): n=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(n, d["wall_ms"], d["outcrc"], "k_match", d["k_match"], "pspec", d["k_pspec"], "pjoin", d["k_pjoin"])
PY

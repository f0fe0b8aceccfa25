#!/bin/bash
# k_emit token loads batched (histogram and packing) A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s10
mkdir -p $O
cd $R
bash tools/variants.sh run base emitb km2 base km2 > $O/var.log 2>&1 || { tail -5 $O/var.log; exit 3; }
python3 - $O/var.log <<'PY'
import sys, json
n=None
for l in open(sys.argv[1]):
    if l.startswith("=="): n=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(n, d["wall_ms"], d["ok"], d["outcrc"], "emit", d["k_emit"], "match", d["k_match"], "pjoin", d["k_pjoin"], "c4", d["k_chains<4>"])
PY

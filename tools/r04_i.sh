#!/bin/bash
# k_inflate_par LDS footprint (waves per CU) A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s9
mkdir -p $O
cd $R
bash tools/variants.sh run p0 pw384 pw256 pw384n2 p0 pw384n2 > $O/var.log 2>&1 || { tail -5 $O/var.log; exit 3; }
python3 - $O/var.log <<'PY'
import sys, json
n=None
for l in open(sys.argv[1]):
    if l.startswith("=="): n=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(n, d["wall_ms"], d["ok"], "par", d["k_inflate_par"], "res", d["k_inflate_resolve"], "infl", d["k_inflate"], "mp", d.get("k_inflate_mp"))
PY

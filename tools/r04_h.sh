#!/bin/bash
# GPU suite (ch3 k_chains in the main library), then waves-per-EU A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s8
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 3; }
bash tools/variants.sh run ch3 wpe0 wpe pj8 wpe0 wpe > $O/var.log 2>&1 || { tail -5 $O/var.log; exit 3; }
python3 - $O/var.log <<'PY'
import sys, json
n=None
for l in open(sys.argv[1]):
    if l.startswith("=="): n=l.split()[1]
    elif l.startswith("{"):
        d=json.loads(l); print(n, d["wall_ms"], d["ok"], d["outcrc"], "c4", d["k_chains<4>"], "c3", d["k_chains<3>"], "pjoin", d["k_pjoin"], "emit", d["k_emit"], "pspec", d["k_pspec"])
PY

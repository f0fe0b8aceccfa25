#!/bin/bash
# GPU suite on the current tree, then timing of the current library
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s7
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 3; }
bash tools/variants.sh run ch3 ch3 > $O/var.log 2>&1 || { tail -5 $O/var.log; exit 3; }
grep "{" $O/var.log | cut -c1-420

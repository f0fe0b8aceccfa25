#!/bin/bash
# session check: GPU suite at HEAD, then k_pspec ring/segment variants
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | head; exit 3; }
bash tools/variants.sh run base w32 w32p8 p8 base 2>&1 | tee $O/var.log

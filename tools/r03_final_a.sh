#!/bin/bash
# full GPU suite and smoke (round-3 final evidence, part a)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_final
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | head; exit 3; }
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 3; }
tail -1 $O/smoke.log

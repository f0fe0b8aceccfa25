#!/bin/bash
# full GPU suite, smoke, then the round's C2+C3 evidence: profiles/collect.sh r03
# (kernel trace + FETCH/WRITE passes) and the default bench line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_main
mkdir -p $O
cd $R
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | head; exit 3; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
bash $R/profiles/collect.sh r03 pmc_summary.json || exit 3
cd $R
timeout -k 10 900 python bench.py > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench.log; exit 3; }
tail -1 $O/bench.log

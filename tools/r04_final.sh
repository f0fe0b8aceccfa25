#!/bin/bash
# round-3 session-2 evidence: GPU suite + smoke, kernel trace and FETCH/WRITE
# passes of the bench command (profiles/collect.sh), the default bench line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_final
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | head; exit 3; }
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
bash $R/profiles/collect.sh r04 pmc_summary.json || exit 3
cd $R
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench.log; exit 3; }
tail -1 $O/bench.log | cut -c1-400

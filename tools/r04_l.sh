#!/bin/bash
# suite + C5 and C2+C3 bench lines at HEAD (k_pspec ring restaging off)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_l
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -1 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | head; exit 3; }
timeout -k 10 900 python bench.py --corpus mixed --level 9 --size 4294967296 --steps 3 --warmup 1 --no-cpu --no-host-api > $O/c5.log 2>&1 || { echo "c5 rc=$?"; tail -5 $O/c5.log; exit 3; }
tail -1 $O/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5', d['value'], d['ms_per_step'], d['config']['kernel_ms_per_step']['k_pspec'])"
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench.log; exit 3; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2C3', d['value'], d['ms_per_step'], d['config']['kernel_ms_per_step'])"

#!/bin/bash
# C5 (4 GiB mixed entropy, level 9) bench line at HEAD
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_c5
mkdir -p $O
cd $R
timeout -k 10 900 python bench.py --corpus mixed --level 9 --size 4294967296 --steps 3 --warmup 1 --no-cpu --no-host-api > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench.log; exit 3; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d['config']['kernel_ms_per_step']), json.dumps(d['roofline']))"

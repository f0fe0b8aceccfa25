#!/bin/bash
# Round-2 large-config evidence on the GPU box: C5 and the C4 shard as tests,
# then the C5 bench line under rocprofv3 kernel trace, then the 8 GiB shard bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02_large
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread \
  -k "c5_level9 or c4_shard" > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -20 $O/pytest.log; exit 3; }
tail -3 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt_c5 -o run --output-format csv \
  -- python3 $R/bench.py --corpus mixed --level 9 --size $((4<<30)) --steps 3 --warmup 1 --no-host-api \
  > $O/bench_c5.log 2>&1 || { echo "c5 rc=$?"; tail -5 $O/bench_c5.log; exit 3; }
tail -1 $O/bench_c5.log
timeout -k 10 600 python3 $R/bench.py --size $((8<<30)) --steps 3 --warmup 1 --no-host-api --no-cpu \
  > $O/bench_8g.log 2>&1 || { echo "8g rc=$?"; tail -5 $O/bench_8g.log; exit 3; }
tail -1 $O/bench_8g.log

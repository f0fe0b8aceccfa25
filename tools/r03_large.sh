#!/bin/bash
# Round-3 large-config evidence on the GPU box: the C5 test, the C5 bench
# under rocprofv3 (kernel trace + FETCH_SIZE + WRITE_SIZE passes ->
# profiles/r03_c5_kernel_stats.csv, pmc_summary_c5.json), then the C5 bench
# line itself (with traffic) and the 8 GiB C4-shard bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_large
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread \
  -k "c5_level9 or c4_shard" > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -20 $O/pytest.log; exit 3; }
tail -2 $O/pytest.log
bash $R/profiles/collect.sh r03_c5 pmc_summary_c5.json --corpus mixed --level 9 --size $((4<<30)) || exit 3
cd $R
timeout -k 10 600 python3 $R/bench.py --corpus mixed --level 9 --size $((4<<30)) --steps 3 --warmup 1 --no-host-api \
  > $O/bench_c5.log 2>&1 || { echo "c5 rc=$?"; tail -5 $O/bench_c5.log; exit 3; }
tail -1 $O/bench_c5.log
timeout -k 10 600 python3 $R/bench.py --size $((8<<30)) --steps 3 --warmup 1 --no-host-api --no-cpu \
  > $O/bench_8g.log 2>&1 || { echo "8g rc=$?"; tail -5 $O/bench_8g.log; exit 3; }
tail -1 $O/bench_8g.log

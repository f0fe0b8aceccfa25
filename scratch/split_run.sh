#!/bin/bash
# dev: split-parse parity + timing vs the lane parse
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "split or golden or edge" > gpurun_out/split_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/split_tests.log; exit 3; }
tail -2 gpurun_out/split_tests.log
for mode in lane split; do
  JD_PARSE=$mode timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-host-api > gpurun_out/b_$mode.log 2>&1 || { echo "bench $mode rc=$?"; tail -5 gpurun_out/b_$mode.log; exit 3; }
  python -c "import json,sys; l=[json.loads(x) for x in open('gpurun_out/b_$mode.log') if x.startswith('{')][-1]; print('$mode', l['value'], l['config']['roundtrip_ok'], l['config']['kernel_ms_per_step'])"
done
for mode in lane split; do
  JD_PARSE=$mode timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-host-api --corpus mixed --level 9 > gpurun_out/m_$mode.log 2>&1 || { echo "bench mixed $mode rc=$?"; tail -5 gpurun_out/m_$mode.log; exit 3; }
  python -c "import json,sys; l=[json.loads(x) for x in open('gpurun_out/m_$mode.log') if x.startswith('{')][-1]; print('mixed9 $mode', l['value'], l['config']['roundtrip_ok'], l['config']['kernel_ms_per_step'])"
done

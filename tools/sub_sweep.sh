#!/bin/bash
# bench sweep over the pipelining sub-chunk size (JD_SUB blocks; 0 = off)
mkdir -p gpurun_out
for s in ${SUBS:-0 4096}; do
  JD_SUB=$s timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --no-host-api > gpurun_out/sub_$s.log 2>&1 || { echo "sub $s rc=$?"; exit 3; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sub_$s.log').read().strip().splitlines()[-1]); print('sub', $s, d['value'], d['ms_per_step'], d['config']['kernel_ms_per_step'])"
done

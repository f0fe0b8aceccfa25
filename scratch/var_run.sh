#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 30 ./scratch/scan_test || exit 3
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "split or golden or edge or block_sizes" > gpurun_out/split_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/split_tests.log; exit 3; }
tail -1 gpurun_out/split_tests.log
bash scratch/variants.sh run "$@"

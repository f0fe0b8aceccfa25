#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u scratch/pj_stats2.py > gpurun_out/pj_stats2.log 2>&1; echo rc=$?
bash scratch/split_run.sh

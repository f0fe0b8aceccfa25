#!/bin/bash
# Kernel trace of the drop-in streaming inflate (tools/stream_rate.py on SIZE
# bytes): per-kernel launch counts and durations behind dropin_stream_pcie.
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/stream_prof
mkdir -p $OUT
export SIZE=${SIZE:-$((8<<20))}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/tools/stream_rate.py > $OUT/run.log 2>&1 || { echo "failed $?"; exit 3; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
cat $OUT/run.log | tail -3
head -12 "$f"

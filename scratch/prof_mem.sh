#!/bin/bash
# memory-path counters for the deflate/inflate kernels (256 MiB, 1 rep)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_mem
mkdir -p $OUT
export SIZE=$((256<<20)) REPS=1
timeout -k 10 300 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/a -o run --output-format csv -- python3 $R/scratch/prof_work.py > $OUT/a.log 2>&1 || { echo "a failed $?"; exit 3; }
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TD_BUSY_avr SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_WAVES -d $OUT/b -o run --output-format csv -- python3 $R/scratch/prof_work.py > $OUT/b.log 2>&1 || { echo "b failed $?"; exit 3; }
echo done

#!/bin/bash
# issue-rate counters for the deflate/inflate kernels (256 MiB, 1 rep)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_issue
mkdir -p $OUT
export SIZE=$((256<<20)) REPS=1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES -d $OUT/a -o run --output-format csv -- python3 $R/scratch/prof_work.py > $OUT/a.log 2>&1 || { echo "a failed $?"; exit 3; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/b -o run --output-format csv -- python3 $R/scratch/prof_work.py > $OUT/b.log 2>&1 || { echo "b failed $?"; exit 3; }
echo done

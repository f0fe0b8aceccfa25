#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_issue2
mkdir -p $OUT
export SIZE=$((256<<20)) REPS=1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $OUT/a -o run --output-format csv -- python3 $R/scratch/prof_work.py > $OUT/a.log 2>&1 || { echo "a failed $?"; exit 3; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS -d $OUT/b -o run --output-format csv -- python3 $R/scratch/prof_work.py > $OUT/b.log 2>&1 || { echo "b failed $?"; exit 3; }
echo done

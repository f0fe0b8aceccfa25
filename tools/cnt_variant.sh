#!/bin/bash
# SQ counters for k_match of one variant library: tools/cnt_variant.sh NAME
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
N=$1
OUT=$R/gpurun_out/cnt_$N
mkdir -p $OUT
export SIZE=$((256<<20)) REPS=1 JDAMD_LIB=$R/tools/var/$N/libjdeflate_amd.so
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d $OUT/a -o run --output-format csv -- python3 $R/tools/prof_work.py > $OUT/a.log 2>&1 || { echo "a failed $?"; exit 3; }
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH -d $OUT/b -o run --output-format csv -- python3 $R/tools/prof_work.py > $OUT/b.log 2>&1 || { echo "b failed $?"; exit 3; }
python3 $R/tools/issue_summary.py $OUT | grep k_match

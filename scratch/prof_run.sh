#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $R/scratch/prof_work.py > $OUT/kt.log 2>&1 || { echo "kt failed $?"; exit 3; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc1 -o run --output-format csv -- python3 $R/scratch/prof_work.py > $OUT/pmc1.log 2>&1 || { echo "pmc1 failed $?"; exit 3; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d $OUT/pmc2 -o run --output-format csv -- python3 $R/scratch/prof_work.py > $OUT/pmc2.log 2>&1 || { echo "pmc2 failed $?"; exit 3; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc3 -o run --output-format csv -- python3 $R/scratch/prof_work.py > $OUT/pmc3.log 2>&1 || { echo "pmc3 failed $?"; exit 3; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc4 -o run --output-format csv -- python3 $R/scratch/prof_work.py > $OUT/pmc4.log 2>&1 || { echo "pmc4 failed $?"; exit 3; }
echo done

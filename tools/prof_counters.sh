#!/bin/bash
# SQ issue counters per kernel on tools/prof_work.py (SIZE bytes, 1 rep).
# Usage (GPU box, repo root): bash tools/prof_counters.sh [tag]
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/prof_cnt${1:-}
mkdir -p $OUT
export SIZE=${SIZE:-$((256<<20))} REPS=1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d $OUT/a -o run --output-format csv -- python3 $R/tools/prof_work.py > $OUT/a.log 2>&1 || { echo "a failed $?"; exit 3; }
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH -d $OUT/b -o run --output-format csv -- python3 $R/tools/prof_work.py > $OUT/b.log 2>&1 || { echo "b failed $?"; exit 3; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/c -o run --output-format csv -- python3 $R/tools/prof_work.py > $OUT/c.log 2>&1 || { echo "c failed $?"; exit 3; }
python3 $R/tools/issue_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
python3 $R/tools/sq_json.py $OUT "${SQTAG:-sq}" "$SIZE" "${LEVEL:-6}" "${CORPUS:-text}" > $OUT/sq_summary.json

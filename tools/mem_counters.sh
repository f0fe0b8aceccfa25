#!/bin/bash
# Vector-memory path counters per kernel (L1/TA/TD) on tools/prof_work.py, two
# passes within the per-block limits (4 TCP, 2 TA, 2 TD).
# Usage (GPU box, repo root): bash tools/mem_counters.sh [tag]
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/mem_cnt${1:-}
mkdir -p $OUT
export SIZE=${SIZE:-$((256<<20))} REPS=1
timeout -s KILL 240 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum -d $OUT/c -o run --output-format csv -- python3 $R/tools/prof_work.py > $OUT/c.log 2>&1 || { echo "c failed $?"; exit 3; }
timeout -s KILL 240 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE -d $OUT/d -o run --output-format csv -- python3 $R/tools/prof_work.py > $OUT/d.log 2>&1 || { echo "d failed $?"; exit 3; }
python3 - "$OUT" > $OUT/summary.txt <<'PY'
import collections, csv, glob, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(agg.items()):
    print(f"{k[:40]:40s} " + " ".join(f"{n}={v:.3g}" for n, v in sorted(c.items())))
PY
cat $OUT/summary.txt

#!/bin/bash
# LDS / wait counters for k_match of variant libraries (256 MiB text):
#   tools/cnt_lds.sh NAME...   (NAME=base uses tools/var/base)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for N in "$@"; do
    OUT=$R/gpurun_out/lds_$N
    mkdir -p $OUT
    export SIZE=$((256<<20)) REPS=1 JDAMD_LIB=$R/tools/var/$N/libjdeflate_amd.so
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $OUT/a -o run --output-format csv -- python3 $R/tools/prof_work.py > $OUT/a.log 2>&1 || { echo "a failed $?"; tail -5 $OUT/a.log; exit 3; }
    python3 - $OUT <<'PY'
import collections, csv, glob, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in agg.items():
    if "k_match" in k or "k_pspec" in k or "k_inflate_par" in k:
        print(sys.argv[1].split("/")[-1], k[:20], " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
PY
done

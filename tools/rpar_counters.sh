#!/bin/bash
# SQ counters of k_inflate_rpar on the drop-in stream pattern (tools/rpar_time.py's worker)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/rpar_cnt
mkdir -p $OUT
export JD_IS_TRACE=1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $OUT/a -o run --output-format csv -- python3 $R/tools/rpar_time.py > $OUT/a.log 2>&1 || { echo "a failed $?"; exit 3; }
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU -d $OUT/b -o run --output-format csv -- python3 $R/tools/rpar_time.py > $OUT/b.log 2>&1 || { echo "b failed $?"; exit 3; }
python3 - "$OUT" <<'PY'
import collections, csv, glob, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(agg.items()):
    if "rpar" in k or "resume" in k:
        print(f"{k[:40]:40s} " + " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
PY

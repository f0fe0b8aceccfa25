#!/bin/bash
# HBM traffic per kernel of variant libraries (FETCH_SIZE x2 gfx950 correction,
# WRITE_SIZE; separate passes), GB per GiB of input:
#   tools/traffic_variant.sh NAME...   (NAME=base uses the in-tree library)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for N in "$@"; do
    OUT=$R/gpurun_out/traffic_$N
    mkdir -p $OUT
    export SIZE=$((256<<20)) REPS=1
    if [ "$N" = base ]; then unset JDAMD_LIB; else export JDAMD_LIB=$R/tools/var/$N/libjdeflate_amd.so; fi
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $R/tools/prof_work.py > $OUT/fetch.log 2>&1 || { echo "fetch failed $?"; exit 3; }
    timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $R/tools/prof_work.py > $OUT/write.log 2>&1 || { echo "write failed $?"; exit 3; }
    echo "== $N"
    python3 - "$OUT" <<'PY'
import sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "profiles"))
from summarize import per_kernel
o = sys.argv[1]
f = per_kernel(os.path.join(o, "fetch"), "FETCH_SIZE"); w = per_kernel(os.path.join(o, "write"), "WRITE_SIZE")
scale = 4 * 1024 / 1e9          # KiB per 256 MiB launch -> GB per GiB
tr = tw = 0
for k in sorted(set(f) | set(w)):
    if not k.startswith("k_"): continue
    r, wr = f.get(k, 0) * 2 * scale, w.get(k, 0) * scale
    tr += r; tw += wr
    print(f"  {k:24s} read {r:7.2f}  write {wr:7.2f} GB/GiB")
print(f"  {'total':24s} read {tr:7.2f}  write {tw:7.2f}  sum {tr + tw:7.2f}")
PY
done

#!/bin/bash
# k_pspec W=32 ring (2 waves/SIMD) with restaging, miss statistics
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3
mkdir -p $O
cd $R
bash tools/variants.sh run nopf pf w32p8rs nopf pf > $O/var.log 2>&1 || { tail -5 $O/var.log; exit 3; }
grep -v SPSTAT $O/var.log | grep -v amdgpu.ids | cut -c1-400
for n in w32rsst w32p8rsst; do
  JDAMD_LIB=$R/tools/var/$n/libjdeflate_amd.so SIZE=$((256<<20)) timeout -k 10 200 python3 tools/probe.py > $O/st_$n.log 2>&1 || { tail -5 $O/st_$n.log; exit 3; }
  python3 - $O/st_$n.log <<'PY'
import sys, json
it=mw=lm=0
for l in open(sys.argv[1]):
    if l.startswith("SPSTAT"):
        f=l.split(); it+=int(f[4]); mw+=int(f[6]); lm+=int(f[8])
    elif l.startswith("{"): ps=json.loads(l)["k_pspec"]
print(sys.argv[1].split('/')[-1], "pspec", ps, "iters", it, "miss-wave frac %.3f" % (mw/max(it,1)), "lane-miss per lane-iter %.4f" % (lm/max(it*64,1)))
PY
done

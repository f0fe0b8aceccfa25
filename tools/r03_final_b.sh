#!/bin/bash
# round-3 final evidence, part b: C2+C3 kernel trace + FETCH/WRITE passes
# (profiles/collect.sh), the default bench line, and the kernel stats of the
# marker-free stream decode (tools/fsp_rate.py under rocprofv3)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_final
mkdir -p $O
bash $R/profiles/collect.sh r03 pmc_summary.json || exit 3
cd $R
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench.log; exit 3; }
tail -1 $O/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
SIZE=$((256<<20)) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fsp -o run --output-format csv -- python3 $R/tools/fsp_rate.py > $O/fsp.log 2>&1 || { echo "fsp prof rc=$?"; tail -5 $O/fsp.log; exit 3; }
grep MB_s $O/fsp.log | cut -c1-200

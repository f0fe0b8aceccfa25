#!/bin/bash
# Collect the rocprofv3 evidence for the bench workload on the GPU box:
#   kt    kernel trace + stats of `bench.py --steps 5 --warmup 1 --no-cpu --no-host-api`
#   fetch FETCH_SIZE per dispatch (separate pass; x2 gfx950 correction later)
#   write WRITE_SIZE per dispatch (separate pass)
# then summarize into profiles/<tag>_kernel_stats.csv and profiles/pmc_summary.json.
# Usage (from the repo root, on the GPU box): bash profiles/collect.sh r03 [summary.json] [bench args]
#   e.g. bash profiles/collect.sh r03_c5 pmc_summary_c5.json --corpus mixed --level 9 --size 4294967296
set -u
TAG=${1:-r01}
NAME=${2:-pmc_summary.json}
shift 2 2>/dev/null || shift $#
EXTRA="$*"
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu --no-host-api $EXTRA > "$OUT/kt.log" 2>&1 || { echo "kt rc=$?"; exit 3; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-host-api $EXTRA > "$OUT/fetch.log" 2>&1 || { echo "fetch rc=$?"; exit 3; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-host-api $EXTRA > "$OUT/write.log" 2>&1 || { echo "write rc=$?"; exit 3; }
python3 "$R/profiles/summarize.py" "$OUT" "$TAG" "$NAME" "$EXTRA" && echo done

#!/bin/bash
# run GPU steps; stop at the first fault/abort/timeout (exit codes other than 0/1)
mkdir -p gpurun_out
step() {
  local name=$1; shift
  "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    pytest) step pytest_gpu timeout -k 10 900 python -m pytest tests -m gpu -q -x ;;
    pytestall) step pytest_gpu timeout -k 10 900 python -m pytest tests -m gpu -q ;;
    bench) step bench timeout -k 10 500 python bench.py --steps 5 --warmup 1 ;;
    benchfull) step bench timeout -k 10 500 python bench.py ;;
    smoke) step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
  esac
done

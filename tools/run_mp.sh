cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in tree "$@"; do
  if [ $v = tree ]; then unset JDAMD_LIB; else export JDAMD_LIB=$GRAFT_REPO_ROOT/tools/var/$v/libjdeflate_amd.so; fi
  echo "== $v"
  timeout -k 10 300 python3 tools/kind_probe.py > gpurun_out/kind_$v.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/kind_$v.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['kind'], d['ok'], {k: v for k, v in d.items() if k.startswith('k_inflate') or k in ('k_match','k_pspec')})"
done
unset JDAMD_LIB
timeout -k 10 300 python3 tools/probe.py > gpurun_out/probe_tree.log 2>&1 && grep -v amdgpu gpurun_out/probe_tree.log | cut -c1-300
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu.py -m gpu > gpurun_out/t_mp.log 2>&1
rc=$?
tail -4 gpurun_out/t_mp.log
exit $rc

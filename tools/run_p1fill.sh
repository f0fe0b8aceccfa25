cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_bounds.py tests/test_inflator_stream.py -m gpu > gpurun_out/t_p1.log 2>&1
rc=$?
tail -3 gpurun_out/t_p1.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/kind_probe.py > gpurun_out/kind_probe_fill.log 2>&1
rc=$?
grep kind gpurun_out/kind_probe_fill.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['kind'], d['ok'], 'par', d['k_inflate_par'], 'res', d['k_inflate_resolve'])"
exit $rc

cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_inflator_stream.py tests/test_zstrm.py tests/test_gpu.py -m gpu > gpurun_out/t_infl.log 2>&1
rc=$?
tail -5 gpurun_out/t_infl.log
[ $rc -ne 0 ] && exit $rc
SIZE=$((32<<20)) timeout -k 10 300 python -u tools/stream_rate.py > gpurun_out/srate.log 2>&1
rc=$?
cat gpurun_out/srate.log | tail -5
exit $rc

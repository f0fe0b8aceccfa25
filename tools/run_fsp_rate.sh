cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_fsp.py tests/test_inflator_stream.py tests/test_zstrm.py tests/test_gpu.py -m gpu > gpurun_out/t_fsp.log 2>&1
rc=$?
tail -3 gpurun_out/t_fsp.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/fsp_rate.py > gpurun_out/fsp_rate.log 2>&1
rc=$?
cat gpurun_out/fsp_rate.log
[ $rc -ne 0 ] && exit $rc
SIZE=$((32<<20)) timeout -k 10 300 python -u tools/stream_rate.py > gpurun_out/srate.log 2>&1
rc=$?
tail -3 gpurun_out/srate.log
exit $rc

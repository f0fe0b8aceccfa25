cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_fsp.py -m gpu > gpurun_out/t_fsp.log 2>&1
rc=$?
tail -25 gpurun_out/t_fsp.log
exit $rc

# tests/test_bounds.py, then the whole GPU suite on the JD_BOUNDS build (any
# JD_BOUNDS line printed by a kernel is an access past a buffer end)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bounds.py -m gpu > gpurun_out/t_bounds.log 2>&1
rc=$?
tail -5 gpurun_out/t_bounds.log
[ $rc -ne 0 ] && exit $rc
JDAMD_LIB=$GRAFT_REPO_ROOT/jdeflate_amd/lib_dbg/libjdeflate_amd.so timeout -k 10 1000 python -u -m pytest -q -s --timeout 600 --timeout-method thread tests -m gpu > gpurun_out/t_dbgsuite.log 2>&1
rc=$?
tail -3 gpurun_out/t_dbgsuite.log
echo "JD_BOUNDS lines: $(grep -c JD_BOUNDS gpurun_out/t_dbgsuite.log)"
exit $rc

set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_hybrid_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4/hy_tests.log 2>&1; rc=$?
tail -30 gpurun_out/r4/hy_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/hybrid_ab.py --tp 1 2 4 --steps 500 --rounds 3 --trace > gpurun_out/r4/hy_ab.log 2>&1; rc=$?
cat gpurun_out/r4/hy_ab.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_resident_gpu.py -x -v --timeout 120 --timeout-method thread -k "session or probe" > gpurun_out/r4/res_sess.log 2>&1; rc=$?
grep -E "fc[123]|passed|failed|Error" gpurun_out/r4/res_sess.log | tail -20
exit $rc

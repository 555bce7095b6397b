set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r5b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5b/suite.log 2>&1 || { echo SUITE_FAIL; grep -E "FAIL|Error|assert" gpurun_out/r5b/suite.log | tail -30; tail -5 gpurun_out/r5b/suite.log; exit 1; }
tail -1 gpurun_out/r5b/suite.log
timeout -k 10 400 python -u scripts/hybrid_ab.py --tp 1 2 4 --steps 500 --rounds 3 --trace > gpurun_out/r5b/trace.log 2>&1 || { echo TRACE_FAIL; tail -30 gpurun_out/r5b/trace.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5b/trace.log | grep -v "trace wg"

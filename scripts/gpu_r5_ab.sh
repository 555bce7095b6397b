set -o pipefail
mkdir -p gpurun_out/r5p
timeout -k 10 600 python -u -m pytest tests/test_hybrid_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5p/tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAIL|Error|assert" gpurun_out/r5p/tests.log | tail -20; exit 1; }
tail -1 gpurun_out/r5p/tests.log
rm -f gpurun_out/ab.log
timeout -k 10 900 bash ab/run.sh || { echo AB_FAIL; tail -20 gpurun_out/ab.log; exit 1; }
grep -E "==|hybrid  " gpurun_out/ab.log
timeout -k 10 300 python -u scripts/hybrid_ab.py --tp 1 2 4 --steps 500 --rounds 1 --only hybrid --trace > gpurun_out/r5p/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 gpurun_out/r5p/trace.log; exit 1; }
grep -E "wait end|arrive|stream length" gpurun_out/r5p/trace.log

#!/bin/bash
# Round 3, call R: the persistent chain launch (csrc/chain.hip): its tests, the tests pinned to
# the six-kernel chain, and the default bench with the chain on / off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_chain_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3r_chain.log 2>&1
rc=$?
tail -12 gpurun_out/r3r_chain.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert" gpurun_out/r3r_chain.log | head -30; exit 1; }
$T 300 python -u bench.py > gpurun_out/r3r_bench_chain.json 2> gpurun_out/r3r_bench_chain.err || { tail -20 gpurun_out/r3r_bench_chain.err; exit 1; }
cat gpurun_out/r3r_bench_chain.json
$T 300 python -u bench.py --server_chain off > gpurun_out/r3r_bench_off.json 2> gpurun_out/r3r_bench_off.err || { tail -20 gpurun_out/r3r_bench_off.err; exit 1; }
cat gpurun_out/r3r_bench_off.json

#!/bin/bash
# Round 3, call K (final tree): the GEMM routing bench, the whole GPU suite, the default bench, and its rocprofv3 kernel table.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3k2_suite.log 2>&1
rc=$?
tail -3 gpurun_out/r3k2_suite.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/r3k2_suite.log | head -20; tail -40 gpurun_out/r3k2_suite.log; exit 1; }
$T 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3k2_smoke.log 2>&1 || { tail -20 gpurun_out/r3k2_smoke.log; exit 1; }
tail -1 gpurun_out/r3k2_smoke.log
$T 300 python -u bench.py > gpurun_out/r3k2_bench.json 2> gpurun_out/r3k2_bench.err || { tail -20 gpurun_out/r3k2_bench.err; exit 1; }
cat gpurun_out/r3k2_bench.json
$T 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3k2_prof -o prof -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/r3k2_prof.log 2>&1 || { tail -20 gpurun_out/r3k2_prof.log; exit 1; }
f=$(find gpurun_out/r3k2_prof -name '*kernel_stats.csv' | sort | tail -1)
cp "$f" gpurun_out/r3k2_bench_kernel_stats.csv
find gpurun_out/r3k2_prof -name '*.csv' -delete
python scripts/kstats.py gpurun_out/r3k2_bench_kernel_stats.csv | head -24

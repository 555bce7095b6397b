#!/bin/bash
# Round-5 rehearsal of the driver's round-end GPU tiers: the whole GPU suite, smoke(), the
# N = 1 bench at its defaults, and a rocprofv3 kernel table of one bench step (persistent
# epochs as plain launches: rocprofv3 crashes at exit after a cooperative launch).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r5f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r5f/suite.log 2>&1 || { echo SUITE_FAIL; grep -E "FAIL|Error|assert" gpurun_out/r5f/suite.log | tail -30; tail -5 gpurun_out/r5f/suite.log; exit 1; }
tail -1 gpurun_out/r5f/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5f/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r5f/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > gpurun_out/r5f/bench.json 2> gpurun_out/r5f/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r5f/bench.err; exit 1; }
tail -1 gpurun_out/r5f/bench.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp
SL_PERSIST_WORKGROUPS=256 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r5f/prof" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 > "$R/gpurun_out/r5f/prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/gpurun_out/r5f/prof.log"; exit 1; }
echo prof-done

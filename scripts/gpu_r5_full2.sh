#!/bin/bash
# Round-5 rehearsal (OUT = output dir; also profiles the vanilla persistent epoch) of the driver's round-end GPU tiers: the whole GPU suite, smoke(), the
# N = 1 bench at its defaults, and a rocprofv3 kernel table of one bench step (persistent
# epochs as plain launches: rocprofv3 crashes at exit after a cooperative launch).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r5y}
cd "$R" && mkdir -p gpurun_out/$OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/$OUT/suite.log 2>&1 || { echo SUITE_FAIL; grep -E "FAIL|Error|assert" gpurun_out/$OUT/suite.log | tail -30; tail -5 gpurun_out/$OUT/suite.log; exit 1; }
tail -1 gpurun_out/$OUT/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/$OUT/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/$OUT/bench.err; exit 1; }
tail -1 gpurun_out/$OUT/bench.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp
SL_PERSIST_WORKGROUPS=256 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$OUT/prof" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 > "$R/gpurun_out/$OUT/prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/gpurun_out/$OUT/prof.log"; exit 1; }
echo prof-done
# the vanilla persistent epoch as a plain launch under the profiler
SL_PERSIST_WORKGROUPS=256 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$OUT/prof_va" -o run -- \
  python3 "$R/bench.py" --mode vanilla --steps 1 --warmup 0 > "$R/gpurun_out/$OUT/prof_va.log" 2>&1 || { echo PROF_VA_FAIL; tail -20 "$R/gpurun_out/$OUT/prof_va.log"; exit 1; }
echo prof-va-done

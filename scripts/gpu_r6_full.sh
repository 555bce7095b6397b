#!/bin/bash
# Round-6 rehearsal of the driver's round-end GPU tiers: the whole GPU suite, smoke(), the
# N = 1 bench at its defaults, the U-shape bench, and a rocprofv3 kernel table of the
# U-shape bench (persistent epochs as plain launches: rocprofv3 crashes at exit after a
# cooperative launch).  Output under gpurun_out/r6f (or $1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${1:-r6f}
cd "$R" && mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/suite.log 2>&1 || { echo SUITE_FAIL; grep -E "FAIL|Error|assert" $O/suite.log | tail -30; tail -5 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-300
timeout -k 10 300 python bench.py --mode ushape --steps 20 --warmup 5 > $O/bench_ushape.json 2> $O/bench_ushape.err || { echo US_BENCH_FAIL; tail -20 $O/bench_ushape.err; exit 1; }
tail -1 $O/bench_ushape.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp
SL_PERSIST_WORKGROUPS=256 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_us" -o run -- \
  python3 "$R/bench.py" --mode ushape --steps 1 --warmup 0 > "$R/$O/prof_us.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/$O/prof_us.log"; exit 1; }
echo prof-done

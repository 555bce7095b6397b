#!/bin/bash
# Round-6 rehearsal of the driver's round-end GPU tiers after the remote-Alice epochs: the whole GPU
# suite, smoke(), the N = 1 bench at its defaults, the vanilla bench, and a rocprofv3 kernel table of
# the vanilla bench (persistent epochs as plain launches: rocprofv3 crashes at exit after a
# cooperative launch).  Output under gpurun_out/${1:-r6z}.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${1:-r6z}
cd "$R" && mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/suite.log 2>&1 || { echo SUITE_FAIL; grep -E "FAIL|Error|assert" $O/suite.log | tail -30; tail -5 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-300
timeout -k 10 300 python bench.py --mode vanilla --steps 20 --warmup 5 > $O/bench_vanilla.json 2> $O/bench_vanilla.err || { echo VA_BENCH_FAIL; tail -20 $O/bench_vanilla.err; exit 1; }
tail -1 $O/bench_vanilla.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp
SL_PERSIST_WORKGROUPS=256 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_va" -o run -- \
  python3 "$R/bench.py" --mode vanilla --steps 1 --warmup 0 > "$R/$O/prof_va.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/$O/prof_va.log"; exit 1; }
echo prof-done

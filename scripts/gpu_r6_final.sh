#!/bin/bash
# Round-6 closing rehearsal after the concat pinned-row policy: the whole GPU suite, smoke(), the
# N = 1 bench at its defaults, and the concat (ws = 9) and U-shape benches.  Output under
# gpurun_out/${1:-r6_final}.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${1:-r6_final}
cd "$R" && mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/suite.log 2>&1 || { echo SUITE_FAIL; grep -E "FAIL|Error|assert" $O/suite.log | tail -30; tail -5 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { echo BENCH_FAIL; tail -20 $O/bench_n1.err; exit 1; }
tail -1 $O/bench_n1.json | cut -c1-300
timeout -k 10 300 python bench.py --mode concat --world_size 9 --steps 3 --warmup 1 > $O/bench_concat.json 2> $O/bench_concat.err || { echo CBENCH_FAIL; tail -20 $O/bench_concat.err; exit 1; }
tail -1 $O/bench_concat.json | cut -c1-200
timeout -k 10 300 python bench.py --mode ushape --steps 20 --warmup 5 > $O/bench_ushape.json 2> $O/bench_ushape.err || { echo UBENCH_FAIL; tail -20 $O/bench_ushape.err; exit 1; }
tail -1 $O/bench_ushape.json | cut -c1-200

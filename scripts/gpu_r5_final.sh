#!/bin/bash
# Round-5 closing run: the GPU suite, smoke(), the N = 1 headline bench, the ws = 2 vanilla bench
# with and without the persistent epoch, and rocprofv3 byte counters of the vanilla persistent
# kernel (plain launch; one counter group per pass).  Outputs: gpurun_out/$OUT/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r5z}
cd "$R" && mkdir -p gpurun_out/$OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/$OUT/suite.log 2>&1 || { echo SUITE_FAIL; grep -E "FAIL|Error|assert" gpurun_out/$OUT/suite.log | tail -30; tail -5 gpurun_out/$OUT/suite.log; exit 1; }
tail -1 gpurun_out/$OUT/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/$OUT/smoke.log; exit 1; }
echo smoke ok
for spec in "n1:" "va:--mode vanilla --steps 3" "vaoff:--mode vanilla --split_persist off --steps 3"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 600 python bench.py $args > gpurun_out/$OUT/bench_$name.json 2> gpurun_out/$OUT/bench_$name.err || { echo BENCH_FAIL $name; tail -20 gpurun_out/$OUT/bench_$name.err; exit 1; }
  tail -1 gpurun_out/$OUT/bench_$name.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['ms_per_step'], d['config'].get('split_epochs'), d['config'].get('phase_seconds'))"
done
cd /tmp && export TMPDIR=/tmp
for c in ${PMC-FETCH_SIZE WRITE_SIZE}; do
  SL_PERSIST_WORKGROUPS=256 timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/$OUT/pmc_$c" -o va -- \
    python3 "$R/scripts/vanilla_trace.py" --reps 1 --batches 400 > "$R/gpurun_out/$OUT/pmc_$c.log" 2>&1 || { echo PMC_FAIL $c; tail -5 "$R/gpurun_out/$OUT/pmc_$c.log"; exit 1; }
  echo pmc $c done
done

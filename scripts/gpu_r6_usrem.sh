#!/bin/bash
# round 6: the remote-Alice persistent U-shape epoch (scripts/ushape_remote_one_gpu.py) fp32 / bf16
# at B = 16 / 5 and 2 / 4 row groups; the vanilla flush A/B (ab/run.sh, when present); the
# co-located U-shape / vanilla regression tests and the vanilla bench.  A step that faults, aborts
# or times out ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_usrem
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc $rc"; grep -E "rank|PASS|passed|failed|Error|us/step" $O/$name.log | tail -12
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step us16 200 python -u scripts/ushape_remote_one_gpu.py 16 2 fp32
step us16bf 200 python -u scripts/ushape_remote_one_gpu.py 16 2 bf16
step us5bf 200 python -u scripts/ushape_remote_one_gpu.py 5 2 bf16
step us16rg4 200 python -u scripts/ushape_remote_one_gpu.py 16 4 fp32
if [ -f ab/run.sh ]; then step ab 700 bash ab/run.sh; fi
step tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ushape_persist_gpu.py tests/test_golden_modes_gpu.py tests/test_vanilla_persist_gpu.py tests/test_golden_gpu.py tests/test_long_launch_gpu.py -k "ushape or vanilla"
step bench_va 300 python bench.py --mode vanilla --steps 20 --warmup 5 --json_out $O/bench_vanilla.json

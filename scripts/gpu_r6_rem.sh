#!/bin/bash
# round 6: the vanilla forward-pass form A/B (ab/run.sh: direct MFMA-layout loads vs LDS-staged),
# the remote-Alice persistent vanilla epoch (scripts/vanilla_remote_one_gpu.py), the vanilla /
# remote / long-launch tests and the vanilla bench.  A step that faults, aborts or times out ends
# the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_rem
mkdir -p $O
step() {   # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc $rc"; tail -4 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
if [ -f ab/run.sh ]; then step ab 700 bash ab/run.sh; fi
step rem16 150 python -u scripts/vanilla_remote_one_gpu.py 16 64
step rem5 150 python -u scripts/vanilla_remote_one_gpu.py 5 64
step tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vanilla_persist_gpu.py tests/test_split_remote_gpu.py tests/test_golden_gpu.py tests/test_long_launch_gpu.py -k "vanilla or remote"
step bench_va 300 python bench.py --mode vanilla --steps 20 --warmup 5 --json_out $O/bench_vanilla.json

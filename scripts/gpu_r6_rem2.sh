#!/bin/bash
# round 6: forward-pass ring depth A/B on the direct-load form (ab/run.sh), then the remote-Alice
# persistent vanilla epoch at B = 16 / 5 with the control-calibrated comparison
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_rem2
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc $rc"; tail -6 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step ab 700 bash ab/run.sh
step rem16 200 python -u scripts/vanilla_remote_one_gpu.py 16 64
step rem5 200 python -u scripts/vanilla_remote_one_gpu.py 5 64

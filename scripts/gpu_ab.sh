#!/bin/bash
# A/B wall-clock of server-step variants on one box (same process image, back to back).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
: > gpurun_out/ab.log
run() { timeout -k 10 200 python3 scripts/prof_step.py --time "$@" 2>/dev/null | grep path= | sed "s/^/[$*] /" >> gpurun_out/ab.log || { echo "AB_FAIL $*"; exit 1; }; }
for rep in 1 2; do
  run --path lookahead --steps 1600 --tp 8
  run --path lookahead --steps 1600 --tp 8 --variant 5=1
  run --path lookahead --steps 1600 --tp 8 --variant 5=2
  run --path lookahead --steps 800
  run --path lookahead --steps 800 --variant 5=1
  run --path lookahead --steps 800 --variant 5=2
done
cat gpurun_out/ab.log

#!/bin/bash
# rocprofv3 kernel stats of the N=1 headline bench (one process) and of the native-executor
# server epoch at TP shard sizes 1 and 8 (wall-clock us/step too).  -> gpurun_out/prof_n1*/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_n1" -o bench -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 > "$R/gpurun_out/prof_n1.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/gpurun_out/prof_n1.log"; exit 1; }
tail -1 "$R/gpurun_out/prof_n1.log"
python3 "$R/scripts/kstats.py" $(find "$R/gpurun_out/prof_n1" -name "*kernel_stats.csv" | head -1)
cd "$R"
for tp in 1 8; do
  timeout -k 10 300 python3 scripts/prof_step.py --path native --steps 1280 --tp $tp --time 2>/dev/null | grep path= || { echo "TIME_FAIL $tp"; exit 1; }
done

#!/bin/bash
# rocprofv3 of bench.py (whole SISA round) + TP=8-shard server steps (graph vs eager).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_bench" -o bench -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 > "$R/gpurun_out/prof_bench.log" 2>&1 || { echo PROF_BENCH_FAIL; tail -20 "$R/gpurun_out/prof_bench.log"; exit 1; }
tail -1 "$R/gpurun_out/prof_bench.log"
for p in graph lookahead; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_tp8_$p" -o step -- \
    python3 "$R/scripts/prof_step.py" --path $p --steps 320 --tp 8 > "$R/gpurun_out/prof_tp8_$p.log" 2>&1 || { echo "PROF_FAIL tp8 $p"; tail -20 "$R/gpurun_out/prof_tp8_$p.log"; exit 1; }
done
cd "$R" && timeout -k 10 300 python3 scripts/prof_step.py --path graph --steps 1600 --tp 8 --time > gpurun_out/tp8_graph_time.log 2>&1 && \
  timeout -k 10 300 python3 scripts/prof_step.py --path lookahead --steps 1600 --tp 8 --time > gpurun_out/tp8_eager_time.log 2>&1 && \
  timeout -k 10 300 python3 scripts/prof_step.py --path graph --steps 1600 --time > gpurun_out/tp1_graph_time.log 2>&1 && \
  cat gpurun_out/tp8_graph_time.log gpurun_out/tp8_eager_time.log gpurun_out/tp1_graph_time.log

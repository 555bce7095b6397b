#!/bin/bash
# rocprofv3 kernel statistics of Bob's server step (generic / fused / graph), the SISA
# client step and (PROF_TP8=1) a TP=8 shard step.  Summaries -> gpurun_out/prof_*/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for p in ${PROF_PATHS:-generic fused lookahead graph local}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$p" -o step -- \
    python3 "$R/scripts/prof_step.py" --path $p --steps 320 > "$R/gpurun_out/prof_$p.log" 2>&1 || { echo "PROF_FAIL $p"; tail -20 "$R/gpurun_out/prof_$p.log"; exit 1; }
done
[ -n "$PROF_TP8" ] && { timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_tp8" -o step -- \
  python3 "$R/scripts/prof_step.py" --path graph --steps 320 --tp 8 > "$R/gpurun_out/prof_tp8.log" 2>&1 || { echo "PROF_FAIL tp8"; tail -20 "$R/gpurun_out/prof_tp8.log"; exit 1; }; }
echo prof-done

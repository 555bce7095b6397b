#!/bin/bash
# rocprofv3 kernel stats of bench.py in the given modes -> gpurun_out/prof_bench_<mode>/ + summary.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-ushape}; do
  d="$R/gpurun_out/prof_bench_$m"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o b -- \
    python3 "$R/bench.py" --mode $m --steps 2 --warmup 1 > "$d.log" 2>&1 || { echo "PROF_FAIL $m"; tail -20 "$d.log"; exit 1; }
  echo "== $m"; tail -1 "$d.log" | cut -c1-160
  python3 "$R/scripts/kstats.py" $(find "$d" -name "*kernel_stats.csv" | head -1)
done

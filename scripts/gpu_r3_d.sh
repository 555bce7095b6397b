#!/bin/bash
# Round 3, call D: the native split-mode executor — bitwise tests, vanilla / U-shape ws = 2
# benches native vs Python loop, and kernel tables of both modes under the native executor.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_split_native_gpu.py > gpurun_out/r3d_split_tests.log 2>&1 || { tail -60 gpurun_out/r3d_split_tests.log; exit 1; }
tail -8 gpurun_out/r3d_split_tests.log
for m in vanilla ushape; do
  for v in native python; do
    extra=""; [ $v = python ] && extra="--python_epoch"
    $T 300 python -u bench.py --mode $m --world_size 2 --steps 2 --warmup 1 $extra --json_out gpurun_out/r3d_bench_${m}_${v}.json > gpurun_out/r3d_bench_${m}_${v}.log 2>&1 || { tail -20 gpurun_out/r3d_bench_${m}_${v}.log; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r3d_bench_${m}_${v}.json'));print('$m $v', d['value'], d['config']['phase_seconds'])"
  done
done
for m in vanilla ushape; do
  $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3d_prof_$m -o prof -- python3 bench.py --mode $m --world_size 2 --steps 1 --warmup 1 > gpurun_out/r3d_prof_$m.log 2>&1 || { tail -20 gpurun_out/r3d_prof_$m.log; exit 1; }
  f=$(find gpurun_out/r3d_prof_$m -name '*kernel_stats.csv' | head -1)
  cp "$f" gpurun_out/r3d_${m}_kernel_stats.csv
  echo "== $m"; python scripts/kstats.py gpurun_out/r3d_${m}_kernel_stats.csv
done

#!/bin/bash
# Round 3, call E: concurrent frozen-front forwards (bitwise tests), split-mode native tests,
# kernel tables of vanilla / U-shape (ws = 2) under the native split executor.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_multi_front_gpu.py tests/test_split_native_gpu.py > gpurun_out/r3e_tests.log 2>&1 || { tail -60 gpurun_out/r3e_tests.log; exit 1; }
tail -4 gpurun_out/r3e_tests.log
for m in vanilla ushape sisa; do
  ws=2; [ $m = sisa ] && ws=9
  $T 300 python -u bench.py --mode $m --world_size $ws --steps 2 --warmup 1 --json_out gpurun_out/r3e_bench_${m}.json > gpurun_out/r3e_bench_${m}.log 2>&1 || { tail -20 gpurun_out/r3e_bench_${m}.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3e_bench_${m}.json'));print('$m', d['value'], d['config']['phase_seconds'])"
done
for m in vanilla ushape; do
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3e_prof_$m -o prof -- python3 bench.py --mode $m --world_size 2 --steps 1 --warmup 0 > gpurun_out/r3e_prof_$m.log 2>&1 || { tail -20 gpurun_out/r3e_prof_$m.log; exit 1; }
  f=$(find gpurun_out/r3e_prof_$m -name '*kernel_stats.csv' | sort | tail -1)
  cp "$f" gpurun_out/r3e_${m}_kernel_stats.csv
  find gpurun_out/r3e_prof_$m -name '*.csv' -delete
  echo "== $m"; python scripts/kstats.py gpurun_out/r3e_${m}_kernel_stats.csv
done

#!/bin/bash
# Parity-split LDS image layout in the conv kernels: numerics, benches, one SQ LDS counter pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2s_tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAILED|^E " gpurun_out/r2s_tests.log | head -20; tail -5 gpurun_out/r2s_tests.log; exit 1; }
tail -1 gpurun_out/r2s_tests.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --json_out gpurun_out/r2s_bench_n1.json > gpurun_out/r2s_bench_n1.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/r2s_bench_n1.log; exit 1; }
tail -1 gpurun_out/r2s_bench_n1.log | cut -c1-200
for mode in ushape vanilla; do
  timeout -k 10 300 python bench.py --mode $mode --steps 3 --warmup 1 --json_out gpurun_out/r2s_$mode.json > gpurun_out/r2s_$mode.log 2>&1 || { echo MODE_FAIL $mode; tail -20 gpurun_out/r2s_$mode.log; exit 1; }
  tail -1 gpurun_out/r2s_$mode.log | cut -c1-200
done
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/r2s_pmc" -o b -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --server_epochs 1 --num_samples 7000 > "$R/gpurun_out/r2s_pmc.log" 2>&1 || { echo "PMC_FAIL"; tail -20 "$R/gpurun_out/r2s_pmc.log"; exit 1; }
python3 - "$R/gpurun_out/r2s_pmc" <<'PY' > "$R/gpurun_out/r2s_pmc_summary.txt"
import collections, csv, glob, sys
acc = collections.defaultdict(list)
for path in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "")[:55]
        acc[(k, row["Counter_Name"])].append(float(row["Counter_Value"]))
ks = sorted({k for k, _ in acc})
for k in ks:
    vals = {c: sum(v) / len(v) for (kk, c), v in acc.items() if kk == k}
    n = max(len(v) for (kk, c), v in acc.items() if kk == k)
    print(f"{k:55s} n={n:5d} " + " ".join(f"{c}={vals[c]:.0f}" for c in sorted(vals)))
PY
grep "sl::conv" "$R/gpurun_out/r2s_pmc_summary.txt"

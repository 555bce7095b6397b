#!/bin/bash
# One SQ counter pass (LDS bank conflicts / LDS instructions / waves) over a short N=1 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_bench" -o b -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --samples_per_client 512 > "$R/gpurun_out/pmc_bench.log" 2>&1 || { echo "PMC_FAIL"; tail -20 "$R/gpurun_out/pmc_bench.log"; exit 1; }
python3 - "$R/gpurun_out/pmc_bench" <<'PY' > "$R/gpurun_out/pmc_bench_summary.txt"
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
grep "sl::" "$R/gpurun_out/pmc_bench_summary.txt"

#!/bin/bash
# round 6: benches (vanilla ws = 2, the N = 1 headline) + the persistent-epoch tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_bench
mkdir -p $O
timeout -k 10 300 python bench.py --mode vanilla --steps 20 --warmup 5 --json_out $O/bench_vanilla.json > $O/bench_vanilla.log 2>&1 || { echo "vanilla bench rc $?"; exit 1; }
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --json_out $O/bench_n1.json > $O/bench_n1.log 2>&1 || { echo "n1 bench rc $?"; exit 1; }
python - <<'P'
import json
for f in ("gpurun_out/r6_bench/bench_vanilla.json", "gpurun_out/r6_bench/bench_n1.json"):
    r = json.load(open(f))
    print(f, r["value"], r["ms_per_step"], r["config"].get("server_executor"), r["config"].get("validated"), r["config"].get("validation"))
P

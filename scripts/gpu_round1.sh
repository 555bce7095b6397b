#!/bin/bash
# GPU validation: smoke, HIP-vs-torch bench A/B, end-to-end CLI runs, rocprof kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_hip.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_hip.log; exit 1; }
tail -1 gpurun_out/bench_hip.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --kernels torch > gpurun_out/bench_torch.log 2>&1 || { echo BENCHT_FAIL; tail -30 gpurun_out/bench_torch.log; exit 1; }
tail -1 gpurun_out/bench_torch.log
timeout -k 10 300 python split_nn.py --vanilla --world_size 2 --iterations 1 --seed 0 --no_tqdm --datapath /tmp/sl_data --log_dir gpurun_out/logs_vanilla > gpurun_out/cli_vanilla.log 2>&1 || { echo CLI_FAIL; tail -30 gpurun_out/cli_vanilla.log; exit 1; }
grep -E "perf|Accuracy" gpurun_out/logs_vanilla/bob.log
timeout -k 10 300 python split_nn.py --sisa --world_size 2 --server_epochs 1 --seed 0 --no_tqdm --datapath /tmp/sl_data2 --log_dir gpurun_out/logs_sisa > gpurun_out/cli_sisa.log 2>&1 || { echo CLI2_FAIL; tail -30 gpurun_out/cli_sisa.log; exit 1; }
grep -E "perf|Accuracy" gpurun_out/logs_sisa/bob.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_bench" -o bench -- python3 "$R/bench.py" --steps 3 --warmup 1 > "$R/gpurun_out/prof_bench.log" 2>&1 || { echo PROF_FAIL; tail -30 "$R/gpurun_out/prof_bench.log"; exit 1; }
echo "prof ok"
find "$R/gpurun_out/prof_bench" -name "*stats*" | head

#!/bin/bash
# Every protocol through the real CLI at the reference's defaults (world_size 3, 70k
# synthetic MNIST-shaped samples), timing each run.  Logs -> gpurun_out/cli_<mode>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
run() {
  name=$1; shift
  start=$(date +%s%N)
  timeout -k 10 500 python split_nn.py "$@" --seed 0 --no_tqdm --datapath /tmp/sl_data_$name \
    --log_dir gpurun_out/cli_$name > gpurun_out/cli_$name.log 2>&1 || { echo "CLI_FAIL $name"; tail -30 gpurun_out/cli_$name.log; exit 1; }
  end=$(date +%s%N)
  echo "$name: $(( (end - start) / 1000000 )) ms wall (incl. data generation and startup)"
  grep -E "Accuracy over|\[perf\]" gpurun_out/cli_$name/bob.log | tail -8
}
run sisa --sisa
run ushape
run vanilla --vanilla --iterations 2
run control --control --iterations 2
run concat --sisa --concat --concat_unlearn --server_epochs 1
run sisa_ws5 --sisa --world_size 5 --server_epochs 1

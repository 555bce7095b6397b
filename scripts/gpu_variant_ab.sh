#!/bin/bash
# Interleaved bench A/B of one kernel variant slot across modes (bench.py --kernel_variant).
#   SLOT=20 VALS="0 1 0 1" MODES="vanilla:--mode vanilla --steps 2 --warmup 1;..." bash scripts/gpu_variant_ab.sh
# -> gpurun_out/var_ab.log
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out" && cd "$R"
IFS=';' read -r -a SPECS <<< "${MODES:-vanilla:--mode vanilla --steps 2 --warmup 1;ushape:--mode ushape --steps 2 --warmup 1;concat:--mode concat --world_size 9 --steps 1 --warmup 1}"
for spec in "${SPECS[@]}"; do
  name=${spec%%:*}; args=${spec#*:}
  for v in ${VALS:-0 1 0 1}; do
    timeout -k 10 300 python bench.py $args --kernel_variant ${SLOT:-20}=$v > gpurun_out/var_$name.json 2> gpurun_out/var_$name.err || { echo "BENCH_FAIL $name $v"; tail -5 gpurun_out/var_$name.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$name slot${SLOT:-20}=$v', d['value'], d['ms_per_step'])" gpurun_out/var_$name.json | tee -a gpurun_out/var_ab.log
  done
done

#!/bin/bash
# wgrad_group's W / state cache-policy presets (fused.hip pol_aux, variant 21) on the modes
# whose optimizer stream it is: vanilla and U-shape ws = 2, concat ws = 9.  -> gpurun_out/pol/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/pol"
mkdir -p "$O" && cd "$R"
# MODES: ';'-separated name:args specs
IFS=';' read -r -a SPECS <<< "${MODES:-vanilla:--mode vanilla --steps 2 --warmup 1;ushape:--mode ushape --steps 2 --warmup 1;concat:--mode concat --world_size 9 --steps 1 --warmup 1}"
for spec in "${SPECS[@]}"; do
  name=${spec%%:*}; args=${spec#*:}
  for p in ${POLS:-0 1 2 3 4 5 0}; do
    timeout -k 10 300 python bench.py $args --kernel_variant 21=$p > "$O/${name}_$p.json" 2> "$O/${name}_$p.err" || { echo "BENCH_FAIL $name $p"; tail -5 "$O/${name}_$p.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$name pol=$p', d['value'], d['ms_per_step'])" "$O/${name}_$p.json"
  done
done

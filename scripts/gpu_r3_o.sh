#!/bin/bash
# Round 3, call O: bf16 MFMA in the data / weight gradients — numerics tests, then U-shape and
# SISA benches in bf16 and fp32 (interleaved).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_golden_gpu.py tests/test_kernels_gpu.py -k "bf16 or xcd_grouped" > gpurun_out/r3o_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r3o_tests.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/r3o_tests.log; exit 1; }
for r in 1 2; do
  for dt in fp32 bf16; do
    $T 200 python -u bench.py --mode ushape --dtype $dt --steps 2 --warmup 1 > gpurun_out/r3o_ushape_${dt}_$r.json 2> gpurun_out/r3o_err.log || { tail -20 gpurun_out/r3o_err.log; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r3o_ushape_${dt}_$r.json'));print('ushape',d['dtype'],round(d['value']))"
  done
done
for dt in fp32 bf16; do
  $T 300 python -u bench.py --dtype $dt --steps 2 --warmup 1 > gpurun_out/r3o_sisa_${dt}.json 2> gpurun_out/r3o_err.log || { tail -20 gpurun_out/r3o_err.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3o_sisa_${dt}.json'));print('sisa',d['dtype'],round(d['value']))"
done

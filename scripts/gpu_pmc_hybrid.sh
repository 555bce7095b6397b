#!/bin/bash
# Hardware counters of the hybrid persistent epoch (csrc/hybrid.hip) at TP = 1 / 2 / 4: bytes
# fetched from / written past L2 (FETCH_SIZE, WRITE_SIZE) and the L2 hit rate, one counter
# group per run (rocprofv3 does not split passes), each epoch a plain launch of 256 workgroups
# (SL_PERSIST_WORKGROUPS=256).  Then, last (it may end in a SIGSEGV), one kernel-trace run of
# the cooperative launch under Python's faulthandler: the profiler's exit-time crash.
# -> gpurun_out/pmch/ and gpurun_out/pmch/summary.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/pmch"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for tp in 1 2 4; do
  for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $c | tr ' ' '_')
    SL_PERSIST_WORKGROUPS=256 timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$O/pmc_${tag}_tp$tp" -o hy -- \
      python3 "$R/scripts/hybrid_ab.py" --tp $tp --steps 200 --rounds 1 --only hybrid > "$O/pmc_${tag}_tp$tp.log" 2>&1 || { echo "PMC_FAIL $c tp$tp"; tail -20 "$O/pmc_${tag}_tp$tp.log"; exit 1; }
  done
done
python3 "$R/scripts/pmc_summary.py" "$O" > "$O/summary.txt" && grep -E "hybrid|==" "$O/summary.txt"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/coop" -o coop -- \
  python3 -X faulthandler "$R/scripts/hybrid_ab.py" --tp 1 --steps 50 --rounds 1 --only hybrid > "$O/coop.log" 2>&1
echo "coop rc $?"
tail -40 "$O/coop.log"

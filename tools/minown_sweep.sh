#!/bin/bash
# GPU box: C2 at sharded per-rank key counts vs the owner floor (SHP_SW_MINOWN; diagnostics).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/minown.jsonl
for k in ${KEYS:-1250 2500 5000}; do
  for mo in ${MINOWNS:-512 1024}; do
    SHP_SW_MINOWN=$mo timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --latency-batches 0 --keys $k --steps 5 > gpurun_out/mo_${k}_$mo.log 2>&1 || exit $?
    grep '^{' gpurun_out/mo_${k}_$mo.log | sed "s/^{/{\"minown\": $mo, /" >> gpurun_out/minown.jsonl
  done
done

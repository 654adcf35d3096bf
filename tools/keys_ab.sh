#!/bin/bash
# GPU box: C2 at the per-rank key counts of a key-sharded job (10k/N keys), default owner map
# vs SHP_SW_MINOWN=1 (owners from ~20 keys each only).  Output: gpurun_out/keys_ab.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/keys_ab.jsonl
for k in ${KEYS:-1250 2500 5000}; do
  for mo in 1 0; do
    if [ $mo = 1 ]; then export SHP_SW_MINOWN=1; else unset SHP_SW_MINOWN; fi
    timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --latency-batches 0 --keys $k --steps 5 ${BENCH_ARGS} \
      > gpurun_out/keys_${k}_$mo.log 2>&1 || exit $?
    grep '^{' gpurun_out/keys_${k}_$mo.log | sed "s/^{/{\"minown_env\": \"${SHP_SW_MINOWN:-default}\", /" >> gpurun_out/keys_ab.jsonl
    echo "keys $k minown=${SHP_SW_MINOWN:-default} done" >&2
  done
done

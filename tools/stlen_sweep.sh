#!/bin/bash
# GPU box: C2 kernel times vs the sweep's super-tile length (SHP_SW_STLEN; diagnostics).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/stlen.jsonl
for L in ${STLENS:-32768 65536 131072 262144}; do
  SHP_SW_STLEN=$L timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --latency-batches 0 --steps 5 ${BENCH_ARGS} > gpurun_out/stlen_$L.log 2>&1 || exit $?
  grep '^{' gpurun_out/stlen_$L.log | sed "s/^{/{\"stlen\": $L, /" >> gpurun_out/stlen.jsonl
done

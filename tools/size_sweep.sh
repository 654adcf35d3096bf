#!/bin/bash
# GPU box: C2 per-kernel time per event at several batch sizes (does a smaller, cache-resident
# working set change the scatter/solve cost per event?).  Output: gpurun_out/size_sweep.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/size_sweep.jsonl
for n in ${SIZES:-6250000 12500000 25000000 50000000 100000000}; do
  steps=$(( 500000000 / n )); [ $steps -lt 5 ] && steps=5
  timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --latency-batches 0 --events $n --steps $steps --warmup 2 ${BENCH_ARGS} \
    > gpurun_out/size_$n.log 2>&1 || exit $?
  grep '^{' gpurun_out/size_$n.log >> gpurun_out/size_sweep.jsonl
  echo "size $n done" >&2
done

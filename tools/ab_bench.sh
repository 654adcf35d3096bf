#!/bin/bash
# GPU box: same-box A/B of the C2 bench between the in-tree library and AB_LIB (built by
# tools/build_variant.sh), alternating A B A B.  Output: gpurun_out/ab.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
for r in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export SIDDHI_HIP_DIAG_LIB=$AB_LIB; else unset SIDDHI_HIP_DIAG_LIB; fi
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --latency-batches 0 --steps 5 ${BENCH_ARGS} > gpurun_out/ab_${v}_$r.log 2>&1 || exit $?
    grep '^{' gpurun_out/ab_${v}_$r.log | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/ab.jsonl
  done
done

#!/bin/bash
# GPU box: same-box comparison of the C2 bench across several builds of the library, round-robin
# (AB_LIBS="name=path ..."; "new" = the in-tree library).  Output: gpurun_out/ab.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
for r in 1 2; do
  for nv in new=- ${AB_LIBS}; do
    v=${nv%%=*}; lib=${nv#*=}
    if [ "$lib" = - ]; then unset SIDDHI_HIP_DIAG_LIB; else export SIDDHI_HIP_DIAG_LIB=$lib; fi
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --latency-batches 0 --steps 5 ${BENCH_ARGS} > gpurun_out/ab_${v}_$r.log 2>&1 || exit $?
    grep '^{' gpurun_out/ab_${v}_$r.log | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/ab.jsonl
  done
done

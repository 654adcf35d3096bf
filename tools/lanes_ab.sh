#!/bin/bash
# GPU box: general-lane configs (C3', C4) with the in-tree library vs variants (LIBS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/lanes_ab.jsonl
for cfg in "3b 20000000" "4 10000000"; do
  set -- $cfg
  for v in base ${LIBS}; do
    if [ $v = base ]; then unset SIDDHI_HIP_DIAG_LIB; else export SIDDHI_HIP_DIAG_LIB=siddhi_amd/libsiddhi_hip_$v.so; fi
    timeout -k 10 200 python3 -u bench.py --config $1 --events $2 --no-cpu-baseline --latency-batches 0 --steps 3 --warmup 1 > gpurun_out/lanes_${1}_$v.log 2>&1 || exit $?
    grep '^{' gpurun_out/lanes_${1}_$v.log | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/lanes_ab.jsonl
  done
done

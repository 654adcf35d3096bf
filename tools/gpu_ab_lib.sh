#!/bin/bash
# GPU box: A/B of a variant library (VAR=siddhi_amd/<name>.so) against the in-tree one on one bench
# config (ARGS), alternating, two runs each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in base var; do
    if [ $v = var ]; then export SIDDHI_HIP_DIAG_LIB=$VAR; else unset SIDDHI_HIP_DIAG_LIB; fi
    timeout -k 10 300 python3 -u bench.py $ARGS --no-cpu-baseline --no-expanded --latency-batches 0 --steps 8 --warmup 2 > gpurun_out/ab_${v}_$r.log 2>&1 || { tail -20 gpurun_out/ab_${v}_$r.log; exit 1; }
    grep '^{' gpurun_out/ab_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernel_ms_per_launch']; print('$v', round(d['ms_per_step'],3), round(d['value']/1e9,2), {a:round(b,3) for a,b in k.items()})"
  done
done
unset SIDDHI_HIP_DIAG_LIB

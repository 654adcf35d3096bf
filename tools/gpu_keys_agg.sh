#!/bin/bash
# GPU box: k_sw_lean's cost by key count and by the AGG epilogue: C2 (pairs) and C5 (avg) at 10k and
# 100k keys, two runs each, plus the C5 bench at its own 100k keys with SHP_LEAN_MINMAX-free default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in 2 5; do
    for k in 10000 100000; do
      timeout -k 10 300 python3 -u bench.py --config $cfg --keys $k --no-cpu-baseline --latency-batches 0 --steps 6 --warmup 2 > gpurun_out/ka_${cfg}_${k}_$r.log 2>&1 || { tail -20 gpurun_out/ka_${cfg}_${k}_$r.log; exit 1; }
      grep '^{' gpurun_out/ka_${cfg}_${k}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernel_ms_per_launch']; print('c$cfg keys $k', round(d['ms_per_step'],3), round(d['value']/1e9,2), round(d['config']['matches_per_step_gpu0']/1e6,1), 'M matches', {a:round(b,3) for a,b in k.items()})"
    done
  done
done

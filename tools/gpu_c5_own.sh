#!/bin/bash
# GPU box: C5 (100k keys) at 512 owners (SHP_SW_PREFOWN=512: ~196 keys per owner, the scatter's
# rounds write longer runs) against the default 1024, alternating, two runs each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in 1024 512; do
    if [ $v = 512 ]; then export SHP_SW_PREFOWN=512; else unset SHP_SW_PREFOWN; fi
    timeout -k 10 300 python3 -u bench.py --config 5 --no-cpu-baseline --latency-batches 0 --steps 6 --warmup 2 > gpurun_out/c5own_${v}_$r.log 2>&1 || { tail -20 gpurun_out/c5own_${v}_$r.log; exit 1; }
    grep '^{' gpurun_out/c5own_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernel_ms_per_launch']; print('c5 owners $v', round(d['ms_per_step'],3), round(d['value']/1e9,2), {a:round(b,3) for a,b in k.items()})"
  done
done
unset SHP_SW_PREFOWN

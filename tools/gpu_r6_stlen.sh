#!/bin/bash
# GPU box: the sweep's super-tile length (SHP_SW_STLEN, events per scatter workgroup; default 65536) on C2 and C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for l in 65536 32768 49152 98304 131072; do
  for c in 2 5; do
    SHP_SW_STLEN=$l timeout -k 10 200 python3 -u bench.py --config $c --no-cpu-baseline --e2e-steps 0 --latency-batches 0 --no-expanded \
      > gpurun_out/stlen_${l}_$c.log 2>&1 || { tail -5 gpurun_out/stlen_${l}_$c.log; exit 1; }
    grep '^{' gpurun_out/stlen_${l}_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$l', '$c', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in r.get('kernel_ms_per_launch',{}).items()})"
  done
done
done

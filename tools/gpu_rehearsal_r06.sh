#!/bin/bash
# GPU box: the N=8 rehearsal on one GPU (--same-device: an in-process group of 8 ranks on cuda:0) beside
# N=1, 12.5M events per rank per step, C2, on the final round-6 library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for g in 1 8; do
  if [ $g = 1 ]; then a=""; else a="--same-device --gpus 8"; fi
  timeout -k 10 300 python3 -u bench.py $a --events 12500000 --steps 5 --warmup 2 --no-cpu-baseline --no-expanded --latency-batches 0 --e2e-steps 0 > gpurun_out/rehearsal_$g.log 2>&1 || { tail -10 gpurun_out/rehearsal_$g.log; exit 1; }
  grep '^{' gpurun_out/rehearsal_$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rehearsal n=$g', round(d['ms_per_step'],3), 'ms', round(d['value']/1e9,2), 'G/s', d['config']['parallelism'][:40], {a:round(b,3) for a,b in d['roofline'].get('kernel_ms_per_launch',{}).items()})"
done

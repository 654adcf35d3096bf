#!/bin/bash
# GPU box: owner-count A/B for the sweep: C5 (100k keys) at 1024 / 2048 / 4096 owners, C2 (10k) at 1024 / 2048
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
one() {  # tag, env, args
  local tag=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 -u bench.py "$@" --no-cpu-baseline --no-expanded --latency-batches 0 --steps 8 --warmup 2 > gpurun_out/own_$tag.log 2>&1 || { tail -20 gpurun_out/own_$tag.log; exit 1; }
  grep '^{' gpurun_out/own_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernel_ms_per_launch']; print('$tag', round(d['ms_per_step'],3), round(d['value']/1e9,2), {a:round(b,3) for a,b in k.items()})"
}
for r in 1 2; do
  one c5_1024_$r "SHP_X=1" --config 5
  one c5_2048_$r "SHP_SW_PREFOWN=2048" --config 5
  one c5_4096_$r "SHP_SW_PREFOWN=4096" --config 5
  one c2_1024_$r "SHP_X=1" --config 2
  one c2_2048_$r "SHP_SW_MINOWN=2048" --config 2
done

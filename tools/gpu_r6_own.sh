#!/bin/bash
# GPU box: owner-count A/B for the sweep path (C2 at 10k keys, C5 at 100k): SHP_SW_KPO (keys per owner
# target) and SHP_SW_PREFOWN (the owner count the map stops at) against the defaults, twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
one() {  # label, config, env...
  local lab=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 200 python3 -u bench.py --config $cfg --no-cpu-baseline --e2e-steps 0 --latency-batches 0 --no-expanded \
    > gpurun_out/own_$lab.log 2>&1 || { tail -5 gpurun_out/own_$lab.log; return 1; }
  grep '^{' gpurun_out/own_$lab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$lab', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in r.get('kernel_ms_per_launch',{}).items()})"
}
for rep in 1 2; do
  one c5_def 5 A=1 || exit 1
  one c5_own512 5 SHP_SW_PREFOWN=512 || exit 1
  one c5_own2048 5 SHP_SW_PREFOWN=2048 SHP_SW_KPO=20 || exit 1
  one c2_def 2 A=1 || exit 1
  one c2_kpo40 2 SHP_SW_KPO=40 || exit 1
  one c2_kpo10 2 SHP_SW_KPO=10 || exit 1
done

#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_rehearsal_r06.sh || exit 1
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --e2e-steps 0 --latency-batches 0 > gpurun_out/q_c2.log 2>&1 || { tail -5 gpurun_out/q_c2.log; exit 1; }
grep '^{' gpurun_out/q_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3))"

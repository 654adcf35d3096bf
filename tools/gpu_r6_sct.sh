#!/bin/bash
# GPU box: labs tests on the current library, then the owner scatters (k_sw_scatter, k_co_scatter) built
# for four waves a SIMD (libsiddhi_s4.so) against the default on C2, C5, C3'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_r6_labs2.sh || exit 1
for rep in 1 2; do
for v in hip s4; do
  for c in 2 5 3b; do
    SIDDHI_HIP_DIAG_LIB=$PWD/siddhi_amd/libsiddhi_$v.so timeout -k 10 300 python3 -u bench.py --config $c --no-cpu-baseline \
      --e2e-steps 0 --latency-batches 0 --no-expanded > gpurun_out/sct_${v}_$c.log 2>&1 || { tail -5 gpurun_out/sct_${v}_$c.log; exit 1; }
    grep '^{' gpurun_out/sct_${v}_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', '$c', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in r.get('kernel_ms_per_launch',{}).items()})"
  done
done
done

#!/bin/bash
# GPU box: the logical-absent multisplit's segment length (events per wave: 8192 / 16384 default / 32768)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for v in hip seg8 seg32; do
  for d in 0 0.01; do
    SIDDHI_HIP_DIAG_LIB=$PWD/siddhi_amd/libsiddhi_$v.so timeout -k 10 300 python3 -u bench.py --config 4 --disorder $d --no-cpu-baseline \
      --e2e-steps 0 --latency-batches 0 > gpurun_out/seg_${v}_$d.log 2>&1 || { tail -5 gpurun_out/seg_${v}_$d.log; exit 1; }
    grep '^{' gpurun_out/seg_${v}_$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', '$d', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms')"
  done
done
done

#!/bin/bash
# GPU box: the fused logical-absent clock (k_la_seg_clock + k_la_ms_scatter<true>) -- parity tests,
# then C4 (ordered and 1% disorder) A/B against the device-wide scan (SHP_LABS_SCAN_CLOCK=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_labs.py tests/test_flow_clock.py tests/test_staged_ingest.py tests/test_retention.py -m gpu -x -q \
  --timeout 280 --timeout-method thread --durations=5 > gpurun_out/r6_clock_tests.log 2>&1 || { tail -30 gpurun_out/r6_clock_tests.log; exit 1; }
tail -2 gpurun_out/r6_clock_tests.log
for v in fused scan fused scan; do
  for d in 0 0.01; do
    if [ $v = scan ]; then export SHP_LABS_SCAN_CLOCK=1; else unset SHP_LABS_SCAN_CLOCK; fi
    timeout -k 10 300 python3 -u bench.py --config 4 --disorder $d --no-cpu-baseline --e2e-steps 0 --latency-batches 0 \
      > gpurun_out/r6_clock_${v}_${d}.log 2>&1 || { tail -20 gpurun_out/r6_clock_${v}_${d}.log; exit 1; }
    python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/r6_clock_${v}_${d}.log') if l.startswith('{')][0]; print('$v', '$d', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms')"
  done
done
unset SHP_LABS_SCAN_CLOCK

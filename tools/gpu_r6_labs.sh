#!/bin/bash
# GPU box, round 6: k_labs_w's exact blocks -- the labs tests, then C4 ordered and with 1 % disorder.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_labs.py -m gpu -v --timeout 240 --timeout-method thread -x \
  > gpurun_out/r6_labs_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r6_labs_tests.log
grep -E "FAILED|ERROR|Error" gpurun_out/r6_labs_tests.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
for m in c4 c4d; do
  extra=""; [ $m = c4d ] && extra="--disorder 0.01"
  timeout -k 10 300 python -u bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0 \
    --e2e-steps 0 $extra > gpurun_out/r6_bench_$m.json 2> gpurun_out/r6_bench_$m.err || { tail -5 gpurun_out/r6_bench_$m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r6_bench_$m.json'));print('$m', d['value']/1e9, 'G', d['ms_per_step'], 'ms', {k:round(v,3) for k,v in d['roofline']['kernel_ms_per_launch'].items()}, d['config'].get('engine_stats'))"
done

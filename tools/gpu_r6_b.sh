#!/bin/bash
# GPU box, round 6: staged ingest parity, the labs tests, C4 ordered / 1 % disorder, C2 with the end-to-end line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_staged_ingest.py -m gpu -v --timeout 240 --timeout-method thread \
  > gpurun_out/r6_staged_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6_staged_tests.log; grep -E "^FAILED" gpurun_out/r6_staged_tests.log | head
[ $rc -le 1 ] || exit $rc
bash tools/gpu_r6_labs.sh || exit $?
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0 --no-expanded \
  > gpurun_out/r6_bench_e2e.json 2> gpurun_out/r6_bench_e2e.err || { tail -5 gpurun_out/r6_bench_e2e.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r6_bench_e2e.json'));print(d['value'],d['ms_per_step']);print(json.dumps(d['config']['end_to_end'],indent=1))"

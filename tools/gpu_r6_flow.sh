#!/bin/bash
# GPU box, round 6: the flow / clock mirror tests, the count-sequence dead-state case, retention, the
# pipelined host ingest (parity, then the bench's end-to-end line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_flow_clock.py tests/test_cseq.py tests/test_retention.py \
  tests/test_java_binding.py tests/test_staged_ingest.py -m gpu -v --timeout 240 --timeout-method thread \
  > gpurun_out/r6_flow_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r6_flow_tests.log
grep -E "FAILED|ERROR" gpurun_out/r6_flow_tests.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0 --no-expanded \
  > gpurun_out/r6_bench_e2e.json 2> gpurun_out/r6_bench_e2e.err
rc=$?
tail -3 gpurun_out/r6_bench_e2e.err
python -c "import json;d=json.load(open('gpurun_out/r6_bench_e2e.json'));print(d['value'],d['ms_per_step']);print(json.dumps(d['config']['end_to_end'],indent=1))"
exit $rc

#!/bin/bash
# GPU box: count-sequence tests, then C3' bench lines: 12-byte records (default) vs SHP_CSEQ_WIDE.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_cseq.py tests/test_c3_scale.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/cseq_tests.log 2>&1
rc=$?
tail -2 gpurun_out/cseq_tests.log
grep -E "^FAILED|^ERROR|Error" gpurun_out/cseq_tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
for v in narrow wide narrow wide; do
  if [ $v = wide ]; then export SHP_CSEQ_WIDE=1; else unset SHP_CSEQ_WIDE; fi
  timeout -k 10 300 python3 -u bench.py --config 3b --no-cpu-baseline --latency-batches 0 --steps 5 --warmup 2 > gpurun_out/c3b_$v.log 2>&1 || { tail -20 gpurun_out/c3b_$v.log; exit 1; }
  grep '^{' gpurun_out/c3b_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline'].get('kernel_ms_per_launch'); print('$v', round(d['ms_per_step'],3), round(d['value']/1e9,2), {a:round(b,3) for a,b in (k or {}).items()})"
done

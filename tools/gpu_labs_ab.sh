#!/bin/bash
# GPU box: logical-absent tests (record sort default), then C4 bench lines (--path labs): in-tree vs SHP_LABS_V1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_labs.py tests/test_group.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/labs_tests.log 2>&1
rc=$?
tail -2 gpurun_out/labs_tests.log
grep -E "^FAILED|^ERROR|Error" gpurun_out/labs_tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
for v in new v1 new v1; do
  if [ $v = v1 ]; then export SHP_LABS_V1=1; else unset SHP_LABS_V1; fi
  timeout -k 10 300 python3 -u bench.py --config 4 --path labs --no-cpu-baseline --latency-batches 0 --steps 5 --warmup 2 > gpurun_out/c4_$v.log 2>&1 || { tail -20 gpurun_out/c4_$v.log; exit 1; }
  grep '^{' gpurun_out/c4_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline'].get('kernel_ms_per_launch'); print('$v', round(d['ms_per_step'],3), round(d['value']/1e9,2), {a:round(b,3) for a,b in (k or {}).items()})"
done

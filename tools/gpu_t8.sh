#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --maxfail=3 --timeout 200 --timeout-method thread -m gpu tests/test_labs.py > gpurun_out/t8.log 2>&1
rc=$?; tail -3 gpurun_out/t8.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/t8.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --config 4 --path labs --no-cpu-baseline --latency-batches 0 --steps 3 --warmup 1 > gpurun_out/c4_bench.log 2>&1 || { tail -20 gpurun_out/c4_bench.log; exit 1; }
grep '^{' gpurun_out/c4_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C4', d['value']/1e9, d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"

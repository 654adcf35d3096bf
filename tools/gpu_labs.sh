#!/bin/bash
# GPU box: the logical-absent path's tests, then the C4 bench line (opt-in path 4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_labs.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/labs_tests.log 2>&1
rc=$?
tail -15 gpurun_out/labs_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config 4 --path labs --no-cpu-baseline --latency-batches 0 --steps 3 --warmup 1 > gpurun_out/c4_bench.log 2>&1 || { tail -20 gpurun_out/c4_bench.log; exit 1; }
grep '^{' gpurun_out/c4_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C4', d['value']/1e9, d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"

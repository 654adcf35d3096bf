#!/bin/bash
# GPU box: the whole -m gpu suite (one process), then smoke().
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1
rc=$?
tail -5 gpurun_out/full_tests.log
grep -E "^FAILED" gpurun_out/full_tests.log | head -30
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --config 4 --path labs --no-cpu-baseline --latency-batches 0 --steps 3 --warmup 1 > gpurun_out/c4_bench.log 2>&1 || { tail -20 gpurun_out/c4_bench.log; exit 1; }
grep '^{' gpurun_out/c4_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C4', d['value']/1e9, d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
exit $rc

#!/bin/bash
# GPU box: the whole -m gpu suite (one process), smoke(), then the default bench line (C2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1
rc=$?
tail -4 gpurun_out/full_tests.log
grep -E "^FAILED|^ERROR" gpurun_out/full_tests.log | head -30
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c2.log 2>&1 || { tail -20 gpurun_out/bench_c2.log; exit 1; }
grep '^{' gpurun_out/bench_c2.log > gpurun_out/bench_c2.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_c2.json')); print('C2', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('kernel_ms_per_launch'))"
exit $rc

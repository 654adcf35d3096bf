#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_full_scale.py tests/test_c4_scale.py -m gpu -v --timeout 400 --timeout-method thread --durations=8 \
  > gpurun_out/r6_full_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED|call " gpurun_out/r6_full_tests.log | tail -14; tail -1 gpurun_out/r6_full_tests.log
[ $rc -ne 0 ] && grep -B5 -A25 "Error\|assert" gpurun_out/r6_full_tests.log | head -60
exit $rc

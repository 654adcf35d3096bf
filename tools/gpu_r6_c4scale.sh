#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_c4_scale.py -m gpu -v --timeout 280 --timeout-method thread --durations=5 \
  > gpurun_out/r6_c4scale_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED|call " gpurun_out/r6_c4scale_tests.log | tail -12; tail -1 gpurun_out/r6_c4scale_tests.log
[ $rc -ne 0 ] && grep -B5 -A25 "Error\|assert" gpurun_out/r6_c4scale_tests.log | head -60
exit $rc

#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_retention.py -m gpu -v -k pipelined --timeout 280 --timeout-method thread \
  > gpurun_out/r6_ret_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r6_ret_tests.log | tail -12; tail -1 gpurun_out/r6_ret_tests.log
exit $rc

#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest "tests/test_labs.py::test_labs_more_than_4096_waiting_pairs" -m gpu -v --timeout 300 \
  --timeout-method thread --durations=2 > gpurun_out/r6_t4096.log 2>&1; rc=$?
grep -E "PASSED|FAILED|call " gpurun_out/r6_t4096.log; [ $rc -ne 0 ] && tail -30 gpurun_out/r6_t4096.log
exit $rc

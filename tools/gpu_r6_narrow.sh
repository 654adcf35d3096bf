#!/bin/bash
# GPU box: the mirror's pipelined flush, wide and narrow forms, against the oracle
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_flow_clock.py tests/test_staged_ingest.py -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/r6_narrow_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r6_narrow_tests.log | grep -i "pipelined\|FAIL\|ERROR" | tail -20
tail -1 gpurun_out/r6_narrow_tests.log
exit $rc

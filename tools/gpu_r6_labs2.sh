#!/bin/bash
# GPU box: the labs tests on the library whose exact k_labs_w variant is built for four waves a SIMD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_labs.py tests/test_flow_clock.py tests/test_staged_ingest.py -m gpu -q -x --timeout 280 \
  --timeout-method thread > gpurun_out/r6_labs2_tests.log 2>&1 || { tail -30 gpurun_out/r6_labs2_tests.log; exit 1; }
tail -1 gpurun_out/r6_labs2_tests.log

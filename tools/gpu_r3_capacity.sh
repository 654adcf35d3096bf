#!/bin/bash
# GPU box: the capacity tests (spilled sweep owners, labs rings past 4096, lanes past x16), then the
# k_sw_bal A/B (tools/gpu_ab_bal.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_spill.py tests/test_capacity.py tests/test_labs.py tests/test_group.py -m gpu -v -x \
  --timeout 240 --timeout-method thread > gpurun_out/cap_tests.log 2>&1
rc=$?
tail -5 gpurun_out/cap_tests.log
grep -E "^FAILED|^ERROR|Error" gpurun_out/cap_tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_ab_bal.sh

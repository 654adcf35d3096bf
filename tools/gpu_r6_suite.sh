#!/bin/bash
# GPU box: the whole -m gpu suite on the final tree (one process), then smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1150 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 400 --timeout-method thread > gpurun_out/full_tests.log 2>&1
rc=$?
tail -3 gpurun_out/full_tests.log
grep -E "^FAILED|^ERROR" gpurun_out/full_tests.log | head -30
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/smoke.log

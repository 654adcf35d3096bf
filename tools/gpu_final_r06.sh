#!/bin/bash
# GPU box, round 6 final library: bench lines for every config (C2 with its end-to-end line), then the
# whole -m gpu suite (one process) and smoke().  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CONFIGS="${CONFIGS:-c2 c3b c5 c4 c4d c3 c1}" bash tools/gpu_bench_all.sh || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1
rc=$?
tail -4 gpurun_out/full_tests.log
grep -E "^FAILED|^ERROR" gpurun_out/full_tests.log | head -30
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/smoke.log

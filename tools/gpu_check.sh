#!/bin/bash
# One GPU session: parity tests, smoke, short bench. Stops at the first fault/timeout
# (exit >= 124 or signal); plain test failures (exit 1) do not stop the later steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1; shift
  echo "== $name: $*" >&2
  "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -5 "gpurun_out/$name.log" >&2
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "== fault/timeout in $name, stopping" >&2; exit $rc; fi
  return 0
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 300 --timeout-method thread ${PYTEST_ARGS}
step smoke timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench timeout -k 10 400 python -u bench.py ${BENCH_ARGS}
if [ -n "$PROF" ]; then
  export TMPDIR=/tmp
  step prof timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 -u bench.py --no-cpu-baseline --latency-batches 0 ${BENCH_ARGS}
fi
exit 0

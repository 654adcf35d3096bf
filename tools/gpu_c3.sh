#!/bin/bash
# GPU box: the count-sequence tests (TESTS), then C3' bench lines: CHAIN32 by owners, CHAIN32 on the
# sorted records (SHP_CO_OFF=1), FULL.  Each step under its own time limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/c3_tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR|passed|failed" gpurun_out/c3_tests.log | tail -30
  [ $rc -ne 0 ] && exit $rc
fi
summ() {
  grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernel_ms_per_launch']; print('$2', round(d['ms_per_step'],3), round(d['value']/1e9,2), d['config']['engine_path'], {a:round(b,3) for a,b in k.items()})"
}
for v in ${VARIANTS:-own sort full}; do
  args="--config 3b --no-cpu-baseline --latency-batches 0 --steps ${STEPS:-6} --warmup 2 ${BENCH_ARGS}"
  case $v in
    own) unset SHP_CO_OFF ;;
    sort) export SHP_CO_OFF=1 ;;
    full) unset SHP_CO_OFF; args="$args --cseq-layout full" ;;
  esac
  timeout -k 10 300 python3 -u bench.py $args > gpurun_out/c3_$v.log 2>&1 || { tail -20 gpurun_out/c3_$v.log; exit 1; }
  summ gpurun_out/c3_$v.log $v
done
unset SHP_CO_OFF

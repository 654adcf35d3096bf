#!/bin/bash
# GPU box: bench lines for the in-tree library and each library in VARIANTS (space-separated paths),
# alternating, twice.  BENCH_ARGS: bench flags (e.g. --config 3b).  Optional TESTS run first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/var_tests.log 2>&1
  rc=$?
  tail -2 gpurun_out/var_tests.log
  grep -E "^FAILED|^ERROR" gpurun_out/var_tests.log | head
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for r in 1 2; do
  for v in intree $VARIANTS; do
    if [ $v = intree ]; then unset SIDDHI_HIP_DIAG_LIB; else export SIDDHI_HIP_DIAG_LIB=$v; fi
    n=$(basename $v .so)
    timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --latency-batches 0 --steps 5 --warmup 2 ${BENCH_ARGS} > gpurun_out/var_${n}_$r.log 2>&1 || { tail -20 gpurun_out/var_${n}_$r.log; exit 1; }
    grep '^{' gpurun_out/var_${n}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline'].get('kernel_ms_per_launch'); print('$n', round(d['ms_per_step'],3), round(d['value']/1e9,2), {a:round(b,3) for a,b in (k or {}).items()})"
  done
done

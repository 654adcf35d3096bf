#!/bin/bash
# GPU box: TESTS, then bench lines for the in-tree library, each library in VARIANTS and AB_LIB
# (default siddhi_amd/base_r4.so), alternating, REPS times per config in CONFIGS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rc=0
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR|passed|failed" gpurun_out/ab_tests.log | tail -30
  [ $rc -gt 1 ] && exit $rc
fi
for cfg in ${CONFIGS:-2}; do
  for r in ${REPS:-1 2}; do
    for v in intree $VARIANTS ${AB_LIB:-siddhi_amd/base_r4.so}; do
      if [ $v = intree ]; then unset SIDDHI_HIP_DIAG_LIB; else export SIDDHI_HIP_DIAG_LIB=$v; fi
      n=$(basename $v .so)
      timeout -k 10 300 python3 -u bench.py --config $cfg --no-cpu-baseline --latency-batches 0 --steps ${STEPS:-6} --warmup 2 > gpurun_out/ab3_c${cfg}_${n}_$r.log 2>&1 || { tail -20 gpurun_out/ab3_c${cfg}_${n}_$r.log; exit 1; }
      grep '^{' gpurun_out/ab3_c${cfg}_${n}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernel_ms_per_launch']; print('c$cfg $n', round(d['ms_per_step'],3), round(d['value']/1e9,2), {a:round(b,3) for a,b in k.items()})"
    done
  done
done
unset SIDDHI_HIP_DIAG_LIB
exit $rc

#!/bin/bash
# GPU box: sweep parity tests on the in-tree library, then the C2 bench A/B against AB_LIB
# (alternating new / base, same box).  BENCH_ARGS extra bench flags; TESTS (default: the sweep set).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_lean_sweep.py tests/test_spill.py tests/test_unordered_ts.py tests/test_group.py"}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?
tail -2 gpurun_out/ab_tests.log
grep -E "^FAILED|^ERROR" gpurun_out/ab_tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export SIDDHI_HIP_DIAG_LIB=$AB_LIB; else unset SIDDHI_HIP_DIAG_LIB; fi
    timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --latency-batches 0 --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/ab_${v}_$r.log 2>&1 || { tail -20 gpurun_out/ab_${v}_$r.log; exit 1; }
    grep '^{' gpurun_out/ab_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernel_ms_per_launch']; print('$v', round(d['ms_per_step'],3), round(d['value']/1e9,2), {a:round(b,3) for a,b in k.items()})"
  done
done

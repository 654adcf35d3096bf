#!/bin/bash
# GPU box: k_sw_bal (SHP_SW_BAL=1) parity on the sweep tests, then A/B bench lines against k_sw_lean.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SHP_SW_BAL=1 timeout -k 10 600 python -u -m pytest tests/test_lean_sweep.py tests/test_gpu_parity.py -m gpu -q -x \
  -k "lean or sweep or c2 or pairs32 or synthetic or unordered or fallback or far or wide" --timeout 300 --timeout-method thread \
  > gpurun_out/bal_tests.log 2>&1
rc=$?
tail -3 gpurun_out/bal_tests.log
grep -E "^FAILED|^ERROR" gpurun_out/bal_tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 0 1 0 1; do
  SHP_SW_BAL=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-batches 0 --steps 10 --warmup 2 > gpurun_out/ab_bal_$v.log 2>&1 || { tail -20 gpurun_out/ab_bal_$v.log; exit 1; }
  grep '^{' gpurun_out/ab_bal_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernel_ms_per_launch']; print('bal=$v', round(d['ms_per_step'],3), {a:round(b,3) for a,b in k.items()})"
done

#!/bin/bash
# GPU box: scatter with e1's filter typed (default) vs generic doubles (SHP_SCATTER_GENERIC), same box,
# alternating; then the sweep parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --latency-batches 0 > gpurun_out/ab_typed_$r.log 2>&1 || { tail -5 gpurun_out/ab_typed_$r.log; exit 1; }
  SHP_SCATTER_GENERIC=1 timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --latency-batches 0 > gpurun_out/ab_generic_$r.log 2>&1 || { tail -5 gpurun_out/ab_generic_$r.log; exit 1; }
done
for f in gpurun_out/ab_typed_*.log gpurun_out/ab_generic_*.log; do
  grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_launch'].items()})"
done
timeout -k 10 400 python -u -m pytest tests/test_lean_sweep.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ab_tests.log; exit $rc

#!/bin/bash
# GPU box (round 4): the tests touched this session, then C5 at 100k keys with 1024 / 2048 owners.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TESTS:-"tests/test_java_binding.py tests/test_spill.py tests/test_group.py tests/test_lean_sweep.py tests/test_gpu_parity.py::test_c5_minmax_at_100k_keys_on_lean tests/test_gpu_parity.py::test_device_aggregate_vs_oracle_selector tests/test_gpu_parity.py::test_device_minmax_java_nan_and_signed_zero tests/test_gpu_parity.py::test_c5_aggregate_at_100k_keys"}
timeout -k 10 1000 python -u -m pytest $T -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r4_check.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r4_check.log | tail -80
[ $rc -gt 1 ] && exit $rc
for v in 1024 2048; do
  export SHP_SW_PREFOWN=$v
  timeout -k 10 300 python3 -u bench.py --config 5 --no-cpu-baseline --latency-batches 0 --steps 5 --warmup 2 > gpurun_out/c5_own$v.log 2>&1 || { tail -20 gpurun_out/c5_own$v.log; exit 1; }
  grep '^{' gpurun_out/c5_own$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline'].get('kernel_ms_per_launch'); print('own$v', round(d['ms_per_step'],3), round(d['value']/1e9,2), {a:round(b,3) for a,b in (k or {}).items()})"
done
# C2: the tree against AB_LIB (default siddhi_amd/base_r4.so), alternating on this box
AB=${AB_LIB:-siddhi_amd/base_r4.so}
unset SHP_SW_PREFOWN
for r in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export SIDDHI_HIP_DIAG_LIB=$AB; else unset SIDDHI_HIP_DIAG_LIB; fi
    timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --latency-batches 0 --steps 10 --warmup 2 > gpurun_out/c2ab_${v}_$r.log 2>&1 || { tail -20 gpurun_out/c2ab_${v}_$r.log; exit 1; }
    grep '^{' gpurun_out/c2ab_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernel_ms_per_launch']; print('c2 $v', round(d['ms_per_step'],3), round(d['value']/1e9,2), {a:round(b,3) for a,b in k.items()})"
  done
done
unset SIDDHI_HIP_DIAG_LIB
exit $rc

#!/bin/bash
# GPU box (round 3): capacity tests (spilled sweep owners, labs rings past 4096, lanes past x16),
# the group gather, k_sw_lean incl. its AGG fold, then the C5 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_spill.py tests/test_capacity.py tests/test_labs.py tests/test_group.py \
  tests/test_lean_sweep.py "tests/test_gpu_parity.py::test_device_aggregate_vs_oracle_selector" \
  "tests/test_gpu_parity.py::test_device_aggregate_snapshot_restore" -m gpu -v -x \
  --timeout 240 --timeout-method thread > gpurun_out/cap_tests.log 2>&1
rc=$?
tail -5 gpurun_out/cap_tests.log
grep -E "^FAILED|^ERROR|Error" gpurun_out/cap_tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline --latency-batches 0 --steps 10 --warmup 2 > gpurun_out/bench_c5.log 2>&1 || { tail -20 gpurun_out/bench_c5.log; exit 1; }
grep '^{' gpurun_out/bench_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5', d['value']/1e9, d['ms_per_step'], d['roofline'].get('kernel_ms_per_launch'))"

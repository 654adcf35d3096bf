#!/bin/bash
# GPU box: k_sw_lean and k_cseq parity (lean, count-sequence and unordered-ts tests, sweep and
# snapshot subsets of the parity suite, the C3' group), then short C2 and C3' benches and the C2
# rocprof kernel summary.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --maxfail=10 --timeout 300 --timeout-method thread -m gpu \
  tests/test_lean_sweep.py tests/test_cseq.py tests/test_labs.py tests/test_unordered_ts.py \
  "tests/test_gpu_parity.py::test_c2_10k_keys_fast_path_vs_oracle" "tests/test_gpu_parity.py::test_sweep_key_counts_vs_oracle" \
  "tests/test_gpu_parity.py::test_sweep_comparison_grid_vs_oracle" "tests/test_gpu_parity.py::test_pairs32_layout_vs_oracle" \
  "tests/test_gpu_parity.py::test_snapshot_restore_continues_exactly" "tests/test_group.py::test_group_c3b_count_lanes" \
  > gpurun_out/lean_tests.log 2>&1
rc=$?
tail -3 gpurun_out/lean_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/lean_tests.log; exit $rc; fi
timeout -k 10 200 python -u bench.py --no-cpu-baseline --latency-batches 0 ${BENCH_ARGS} > gpurun_out/lean_bench.log 2>&1 || { tail -20 gpurun_out/lean_bench.log; exit 1; }
grep '^{' gpurun_out/lean_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', d['value']/1e9, d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
timeout -k 10 300 python -u bench.py --config 3b --no-cpu-baseline --latency-batches 0 --steps 3 --warmup 1 > gpurun_out/c3b_bench.log 2>&1 || { tail -20 gpurun_out/c3b_bench.log; exit 1; }
grep '^{' gpurun_out/c3b_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3b', d['value']/1e9, d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
timeout -k 10 300 python -u bench.py --config 4 --path labs --no-cpu-baseline --latency-batches 0 --steps 3 --warmup 1 > gpurun_out/c4_bench.log 2>&1 || { tail -20 gpurun_out/c4_bench.log; exit 1; }
grep '^{' gpurun_out/c4_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C4', d['value']/1e9, d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lean_prof -o run -- python3 -u bench.py --no-cpu-baseline --latency-batches 0 ${BENCH_ARGS} > gpurun_out/lean_prof.log 2>&1 || { tail -20 gpurun_out/lean_prof.log; exit 1; }
find gpurun_out/lean_prof -name "*stats*" | head -5

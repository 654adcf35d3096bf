#!/bin/bash
# GPU box: the sweep path (12-byte records) -- parity tests, then C2 / C5 benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lean_sweep.py tests/test_spill.py tests/test_win_sweep.py tests/test_retention.py -m gpu > gpurun_out/r5_sweep_tests.log 2>&1 || { tail -30 gpurun_out/r5_sweep_tests.log; exit 1; }
tail -2 gpurun_out/r5_sweep_tests.log
CONFIGS="${SW_CONFIGS:-c2 c5}" bash tools/gpu_bench_all.sh

#!/bin/bash
# GPU box: logical-absent path -- parity tests, phase stamps, C4 bench (ordered and 1% disorder)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_labs.py -m gpu > gpurun_out/r5_labs_tests.log 2>&1 || { tail -30 gpurun_out/r5_labs_tests.log; exit 1; }
tail -2 gpurun_out/r5_labs_tests.log
SIDDHI_HIP_DIAG_LIB=siddhi_amd/libsiddhi_hip_stamps.so timeout -k 10 300 python3 -u tools/labs_probe.py --reps 2 > gpurun_out/labs_probe.txt 2>&1 || { tail gpurun_out/labs_probe.txt; exit 1; }
tail -11 gpurun_out/labs_probe.txt
CONFIGS="${LABS_CONFIGS:-c4}" bash tools/gpu_bench_all.sh

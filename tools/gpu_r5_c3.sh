#!/bin/bash
# GPU box: the count-sequence modes (cs_tables) -- tests, then C3 / C4 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cseq.py tests/test_c3_scale.py tests/test_chain32.py -m gpu > gpurun_out/r5_c3_tests.log 2>&1 || { tail -30 gpurun_out/r5_c3_tests.log; exit 1; }
tail -3 gpurun_out/r5_c3_tests.log
CONFIGS="c3 c4 c4d" bash tools/gpu_bench_all.sh

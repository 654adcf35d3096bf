#!/bin/bash
# GPU box: lean parity tests, then a same-box A/B of the C2 bench against AB_LIBS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --maxfail=3 --timeout 200 --timeout-method thread -m gpu tests/test_lean_sweep.py \
  "tests/test_gpu_parity.py::test_sweep_comparison_grid_vs_oracle" "tests/test_unordered_ts.py" > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/ab_tests.log | head; exit $rc; fi
bash tools/ab_multi.sh
python3 - <<'P'
import json
for l in open('gpurun_out/ab.jsonl'):
    d = json.loads(l)
    k = d['roofline']['kernel_ms_per_launch']
    print(d['variant'], round(d['ms_per_step'], 3), {a: round(b, 3) for a, b in k.items()})
P

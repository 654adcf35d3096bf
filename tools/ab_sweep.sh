#!/bin/bash
# GPU box: sweep-path parity subset, then a same-box A/B of the C2 bench (in-tree library vs AB_LIB).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_unordered_ts.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -k "sweep or c2 or c5 or pairs32 or aggregate or unordered or default" > gpurun_out/ab_tests.log 2>&1
rc=$?
tail -3 gpurun_out/ab_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/ab_bench.sh
python3 - <<'PY'
import json
for l in open('gpurun_out/ab.jsonl'):
    d = json.loads(l)
    k = d['roofline']['kernel_ms_per_launch']
    print(d['variant'], round(d['ms_per_step'], 3), {a: round(b, 3) for a, b in k.items()})
PY

#!/bin/bash
# GPU box: k_labs_out's interpolated fire search -- labs parity tests, C4 kernel stats, then the sweep
# owner-count A/B (tools/gpu_r6_own.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_labs.py tests/test_flow_clock.py -m gpu -x -q --timeout 280 --timeout-method thread \
  > gpurun_out/r6_out_tests.log 2>&1 || { tail -30 gpurun_out/r6_out_tests.log; exit 1; }
tail -1 gpurun_out/r6_out_tests.log
bash tools/gpu_r6_c4stats.sh || exit 1
python3 -c "
import csv
for v in ['fused','scan']:
    for r in csv.DictReader(open(f'gpurun_out/c4s_{v}/run_kernel_stats.csv')):
        if 'k_labs_out' in r['Name'] or 'k_la_ms' in r['Name'] or 'k_labs_w<true, false>' in r['Name']: print(v, r['Name'][:40], round(float(r['AverageNs'])/1e3,1), 'us')
"
bash tools/gpu_r6_own.sh

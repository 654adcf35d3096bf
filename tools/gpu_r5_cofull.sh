#!/bin/bash
# GPU box: the owner path's FULL rows (k_co_run<., true>) -- parity tests, then C3' / C3 benches both layouts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cseq.py tests/test_c3_scale.py tests/test_chain32.py tests/test_retention.py -m gpu > gpurun_out/r5_cofull_tests.log 2>&1 || { tail -30 gpurun_out/r5_cofull_tests.log; exit 1; }
tail -3 gpurun_out/r5_cofull_tests.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python3 -u bench.py "$@" > gpurun_out/bench_$name.log 2>&1 || { tail -20 gpurun_out/bench_$name.log; return 1; }
  grep '^{' gpurun_out/bench_$name.log > gpurun_out/bench_$name.json
  python3 -c "import json; d=json.load(open('gpurun_out/bench_$name.json')); print('$name', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms', d['config']['match_layout'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_launch'].items()}, 'exp', (d['config'].get('expanded') or {}).get('value'))"
}
run c3bfull --config 3b --cseq-layout full --no-cpu-baseline && run c3b --config 3b --no-cpu-baseline && run c3full --config 3 --cseq-layout full --no-cpu-baseline

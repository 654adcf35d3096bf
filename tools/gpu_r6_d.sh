#!/bin/bash
# GPU box, round 6: staged / narrow ingest parity, the labs default-path tests (tie seeds vs lanes),
# then C2 with the end-to-end line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_staged_ingest.py "tests/test_labs.py::test_labs_default_path_any_order_vs_oracle" \
  -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r6_d_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6_d_tests.log; grep -E "^FAILED" gpurun_out/r6_d_tests.log | head
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0 --no-expanded \
  > gpurun_out/r6_bench_e2e.json 2> gpurun_out/r6_bench_e2e.err || { tail -5 gpurun_out/r6_bench_e2e.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r6_bench_e2e.json'));print(d['value'],d['ms_per_step']);e=d['config']['end_to_end'];print(e['value'],e['mode'],{k:(round(v['value']/1e9,2),round(v['ms_per_step'],1),round(v['pcie_gbs'],1)) for k,v in e['forms'].items()}, e['h2d_copy_gbs'])"

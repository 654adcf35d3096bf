#!/bin/bash
# GPU box: variant library (siddhi_amd/lib_tsmax.so: the push's max ts in k_co_scatter, k_co_count reads
# keys only) -- C3' parity under it, then the C3' / C3 A/B against the in-tree library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=siddhi_amd/lib_tsmax.so
SIDDHI_HIP_DIAG_LIB=$V timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_chain32.py tests/test_c3_scale.py > gpurun_out/tsmax_tests.log 2>&1 || { tail -30 gpurun_out/tsmax_tests.log; exit 1; }
tail -1 gpurun_out/tsmax_tests.log
one() {  # tag, env, args
  local tag=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 -u bench.py "$@" --no-cpu-baseline --no-expanded --latency-batches 0 --steps 10 --warmup 3 > gpurun_out/tsm_$tag.log 2>&1 || { tail -20 gpurun_out/tsm_$tag.log; exit 1; }
  grep '^{' gpurun_out/tsm_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernel_ms_per_launch']; print('$tag', round(d['ms_per_step'],3), round(d['value']/1e9,2), {a:round(b,3) for a,b in k.items()})"
}
for r in 1 2; do
  one c3b_base_$r "SHP_X=1" --config 3b
  one c3b_tsmax_$r "SIDDHI_HIP_DIAG_LIB=$V" --config 3b
done
one c3_base "SHP_X=1" --config 3
one c3_tsmax "SIDDHI_HIP_DIAG_LIB=$V" --config 3

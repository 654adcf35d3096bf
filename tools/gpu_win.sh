#!/bin/bash
# GPU box: k_sw_win first light -- a short C2 bench (hang / fault check), the win tests, then the
# C2 bench A/B against k_sw_lean (SHP_NO_WIN=1), alternating on the same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
summ() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernel_ms_per_launch']; print('$2', round(d['ms_per_step'],3), round(d['value']/1e9,2), {a:round(b,3) for a,b in k.items()})"; }
timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --latency-batches 0 --steps 3 --warmup 1 > gpurun_out/win_first.log 2>&1 || { tail -30 gpurun_out/win_first.log; exit 1; }
summ gpurun_out/win_first.log first
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_win_sweep.py} -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/win_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/win_tests.log | tail -40
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for r in 1 2; do
  for v in win lean; do
    if [ $v = lean ]; then export SHP_NO_WIN=1; else unset SHP_NO_WIN; fi
    timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --latency-batches 0 --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/winab_${v}_$r.log 2>&1 || { tail -20 gpurun_out/winab_${v}_$r.log; exit 1; }
    summ gpurun_out/winab_${v}_$r.log $v
  done
done
exit $rc

#!/bin/bash
# GPU box, end of round 3: the whole -m gpu suite, smoke(), the C2 bench line, then the C3' bench
# line (with its CPU baseline) and its rocprof kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_suite_bench.sh || exit $?
timeout -k 10 400 python -u bench.py --config 3b > gpurun_out/bench_c3b.log 2>&1 || { tail -20 gpurun_out/bench_c3b.log; exit 1; }
grep '^{' gpurun_out/bench_c3b.log > gpurun_out/bench_c3b.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_c3b.json')); print('C3b', d['value']/1e9, d['ms_per_step'], d['roofline'].get('kernel_ms_per_launch'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_c3b -o run -- python3 -u bench.py --config 3b --steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0 > gpurun_out/stats_c3b.log 2>&1 || exit $?
echo done

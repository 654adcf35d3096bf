#!/bin/bash
# GPU box: group (multi-GPU behind the C-ABI) tests, then the bench's N>1 path rehearsed in one
# process on cuda:0 (--same-device), then a short N=1 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_group.py -x -q --timeout 200 --timeout-method thread > gpurun_out/group.log 2>&1 || { tail -30 gpurun_out/group.log; exit 1; }
tail -2 gpurun_out/group.log
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --events 20000000 --steps 4 --warmup 2 > gpurun_out/bench_g2.log 2>&1 || { tail -30 gpurun_out/bench_g2.log; exit 1; }
tail -1 gpurun_out/bench_g2.log | cut -c 1-600
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --latency-batches 0 > gpurun_out/bench_g1.log 2>&1 || { tail -30 gpurun_out/bench_g1.log; exit 1; }
tail -1 gpurun_out/bench_g1.log | cut -c 1-400

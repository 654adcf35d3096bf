#!/bin/bash
# GPU box, end of round 4 (after the last library build): C2 kernel stats + PMC traffic
# (tools/pmc_run.sh -> gpurun_out/pmc.json, keyed to this library's hash), C3' and C5 traffic
# (tools/pmc_cfg.sh), C5 kernel stats, then bench lines with CPU baselines for C2 (default: latency
# on), C3', C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_run.sh > gpurun_out/pmc_run_c2.log 2>&1 || { tail -5 gpurun_out/pmc_run_c2.log; exit 1; }
CFG=3b KEYS=1000000 NO_LV=1 bash tools/pmc_cfg.sh > gpurun_out/pmc_cfg_3b.log 2>&1 || { tail -5 gpurun_out/pmc_cfg_3b.log; exit 1; }
CFG=5 KEYS=100000 NO_LV=1 bash tools/pmc_cfg.sh > gpurun_out/pmc_cfg_5.log 2>&1 || { tail -5 gpurun_out/pmc_cfg_5.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_c5 -o run -- python3 -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0 > gpurun_out/stats_c5.log 2>&1 || { tail -5 gpurun_out/stats_c5.log; exit 1; }
cp gpurun_out/pmc.json profiles/pmc_traffic_c2.json
cp gpurun_out/pmc_3b_traffic.json profiles/pmc_traffic_c3b.json
cp gpurun_out/pmc_5_traffic.json profiles/pmc_traffic_c5.json
CONFIGS="c2 c3b c5" bash tools/gpu_bench_all.sh

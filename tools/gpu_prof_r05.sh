#!/bin/bash
# GPU box, round 5 measurement on the final library: rocprof kernel stats for C2, C3', C4, C5 and
# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) for the same configs.  Each step under its own
# limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--steps 3 --warmup 1 --no-cpu-baseline --no-expanded --latency-batches 0"
for c in 2 3b 4 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_c$c -o run -- python3 -u bench.py --config $c $Q > gpurun_out/stats_c$c.log 2>&1 || { tail -5 gpurun_out/stats_c$c.log; exit 1; }
  echo "stats c$c done"
done
BENCH_ARGS="--no-expanded" bash tools/pmc_run.sh > gpurun_out/pmc_run_c2.log 2>&1 || { tail -5 gpurun_out/pmc_run_c2.log; exit 1; }
echo "pmc c2 done"
for c in 3b 4 5; do
  k=1000000; [ $c = 4 ] && k=1000; [ $c = 5 ] && k=100000
  BENCH_ARGS="--no-expanded" NO_LV=1 CFG=$c KEYS=$k bash tools/pmc_cfg.sh > gpurun_out/pmc_cfg_$c.log 2>&1 || { tail -5 gpurun_out/pmc_cfg_$c.log; exit 1; }
  echo "pmc c$c done"
done
echo done

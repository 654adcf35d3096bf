#!/bin/bash
# GPU box, round 6 measurement on the final library: rocprof kernel stats for C2, C3', C4 (ordered
# and 1 % disorder), C5; PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) for the same configs and
# the LDS / VALU / wait counters for C2 and C3'.  Each step under its own limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--steps 3 --warmup 1 --no-cpu-baseline --no-expanded --latency-batches 0 --e2e-steps 0"
for c in 2 3b 4 5 4d; do
  a="--config $c"; [ $c = 4d ] && a="--config 4 --disorder 0.01"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_c$c -o run -- python3 -u bench.py $a $Q > gpurun_out/stats_c$c.log 2>&1 || { tail -5 gpurun_out/stats_c$c.log; exit 1; }
  echo "stats c$c done"
done
BENCH_ARGS="--no-expanded" bash tools/pmc_run.sh > gpurun_out/pmc_run_c2.log 2>&1 || { tail -5 gpurun_out/pmc_run_c2.log; exit 1; }
echo "pmc c2 done"
for c in 3b 4 5; do
  k=1000000; [ $c = 4 ] && k=1000; [ $c = 5 ] && k=100000
  BENCH_ARGS="--no-expanded" NO_LV=1 CFG=$c KEYS=$k bash tools/pmc_cfg.sh > gpurun_out/pmc_cfg_$c.log 2>&1 || { tail -5 gpurun_out/pmc_cfg_$c.log; exit 1; }
  [ $c = 4 ] && cp gpurun_out/pmc_4_traffic.json gpurun_out/pmc_4o_traffic.json  # (the 4d pass below rewrites it)
  echo "pmc c$c done"
done
BENCH_ARGS="--no-expanded --disorder 0.01" NO_LV=1 CFG=4 KEYS=1000 PMC_DISORDER=0.01 bash tools/pmc_cfg.sh > gpurun_out/pmc_cfg_4d.log 2>&1 || { tail -5 gpurun_out/pmc_cfg_4d.log; exit 1; }
mv gpurun_out/pmc_4_traffic.json gpurun_out/pmc_4d_traffic.json
echo "pmc c4d done"
for c in 2 3b; do
  k=10000; [ $c = 3b ] && k=1000000
  BENCH_ARGS="--no-expanded" NO_TRAFFIC=1 CFG=$c KEYS=$k bash tools/pmc_cfg.sh > gpurun_out/pmc_lv_$c.log 2>&1 || { tail -5 gpurun_out/pmc_lv_$c.log; exit 1; }
  echo "lds/valu c$c done"
done
echo done

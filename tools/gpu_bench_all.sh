#!/bin/bash
# GPU box: bench lines (with CPU baselines) for every SURVEY §8d config on its default path
# (C4's is the logical-absent automaton since round 5), and C3 as specified.  CONFIGS overrides the list; each line lands in
# gpurun_out/bench_<name>.json.  Stops at the first failing run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python3 -u bench.py "$@" > gpurun_out/bench_$name.log 2>&1 || { tail -20 gpurun_out/bench_$name.log; return 1; }
  grep '^{' gpurun_out/bench_$name.log > gpurun_out/bench_$name.json
  python3 -c "import json; d=json.load(open('gpurun_out/bench_$name.json')); c=d['cpu_baseline'] or {}; print('$name', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms', d['config']['engine_path'][:60], 'frac', round(d['roofline']['frac'],3), 'cpu', c.get('value'))"
}
for c in ${CONFIGS:-c3b c5 c4 c3 c1}; do
  case $c in
    c2) run c2 400 ;;
    c3b) run c3b 400 --config 3b ;;
    c3bfull) run c3bfull 400 --config 3b --cseq-layout full --no-cpu-baseline ;;
    c5) run c5 400 --config 5 ;;
    c4) run c4 500 --config 4 ;;
    c4d) run c4d 500 --config 4 --disorder 0.01 --no-cpu-baseline --e2e-steps 0 --pmc profiles/pmc_traffic_c4d_0.01.json ;;
    c4lanes) run c4lanes 700 --config 4 --path general --steps 2 --warmup 1 --latency-batches 0 ;;
    c3) run c3 400 --config 3 ;;
    c1) run c1 500 --config 1 --steps 3 --warmup 1 ;;
  esac || exit 1
done

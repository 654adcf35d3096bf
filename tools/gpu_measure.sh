#!/bin/bash
# GPU box: the round's measurement set: C2 kernel stats + PMC traffic, the full C2 bench line
# (roofline with that traffic, CPU baselines, latency), LDS/VALU counters, and the other configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/pmc_run.sh > gpurun_out/pmc_run.log 2>&1 || { tail -20 gpurun_out/pmc_run.log; exit 1; }
echo "pmc traffic done"
timeout -k 10 400 python -u bench.py --pmc gpurun_out/pmc.json > gpurun_out/bench_c2.log 2>&1 || { tail -20 gpurun_out/bench_c2.log; exit 1; }
grep '^{' gpurun_out/bench_c2.log > gpurun_out/bench_c2.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_c2.json')); print('C2', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d['roofline']['step']['frac'], d['roofline']['traffic'])"
bash tools/pmc_c2.sh > gpurun_out/pmc_c2.log 2>&1 || { tail -20 gpurun_out/pmc_c2.log; exit 1; }
echo "pmc lds/valu done"
for c in "1" "3b" "5"; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --latency-batches 0 > gpurun_out/bench_c$c.log 2>&1 || { tail -20 gpurun_out/bench_c$c.log; exit 1; }
  grep '^{' gpurun_out/bench_c$c.log > gpurun_out/bench_c$c.json
  python3 -c "import json; d=json.load(open('gpurun_out/bench_c$c.json')); print('C$c', d['value']/1e9, d['ms_per_step'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
done
timeout -k 10 400 python -u bench.py --config 4 --path labs --steps 3 --warmup 1 --latency-batches 0 > gpurun_out/bench_c4.log 2>&1 || { tail -20 gpurun_out/bench_c4.log; exit 1; }
grep '^{' gpurun_out/bench_c4.log > gpurun_out/bench_c4.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_c4.json')); print('C4', d['value']/1e9, d['ms_per_step'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_c4 -o run -- python3 -u bench.py --config 4 --path labs --steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0 > gpurun_out/stats_c4.log 2>&1 || { tail -20 gpurun_out/stats_c4.log; exit 1; }
echo "c4 stats done"

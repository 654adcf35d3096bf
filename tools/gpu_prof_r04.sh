#!/bin/bash
# GPU box, round 4 measurement: rocprof kernel stats (C2, C3'), PMC traffic (C2 via tools/pmc_run.sh,
# C3' via tools/pmc_cfg.sh), and the N=8 rehearsal on one GPU (--same-device) beside N=1 at the
# same events per rank.  Each step under its own limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_c3b -o run -- python3 -u bench.py --config 3b $Q > gpurun_out/stats_c3b.log 2>&1 || exit $?
bash tools/pmc_run.sh > gpurun_out/pmc_run_c2.log 2>&1 || { tail -5 gpurun_out/pmc_run_c2.log; exit 1; }
CFG=3b KEYS=1000000 bash tools/pmc_cfg.sh > gpurun_out/pmc_cfg_3b.log 2>&1 || { tail -5 gpurun_out/pmc_cfg_3b.log; exit 1; }
for g in 1 8; do
  if [ $g = 1 ]; then a=""; else a="--same-device --gpus 8"; fi
  timeout -k 10 300 python3 -u bench.py $a --events 12500000 --steps 5 --warmup 2 --no-cpu-baseline --latency-batches 0 > gpurun_out/rehearsal_$g.log 2>&1 || { tail -10 gpurun_out/rehearsal_$g.log; exit 1; }
  grep '^{' gpurun_out/rehearsal_$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rehearsal n=$g', round(d['ms_per_step'],3), 'ms', round(d['value']/1e9,2), 'G/s', d['config']['parallelism'][:40])"
done
echo done

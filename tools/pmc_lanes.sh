#!/bin/bash
# GPU box: one rocprofv3 --pmc pass (<= 8 SQ counters) over a short bench of a general-lane
# config; prints per-kernel counter sums.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_lanes
mkdir -p $OUT
timeout -s KILL 150 rocprofv3 --pmc ${COUNTERS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR} --output-format csv -d $OUT -o p -- python3 -u bench.py --config ${CFG:-3b} --events ${EVENTS:-20000000} --no-cpu-baseline --latency-batches 0 --steps 1 --warmup 0 > $OUT/log.txt 2>&1 || exit $?
python3 - <<'PY' > gpurun_out/pmc_lanes.txt
import csv, glob, collections
agg = collections.defaultdict(dict)
for f in glob.glob('gpurun_out/pmc_lanes/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0][-40:]
        agg[k][r['Counter_Name']] = agg[k].get(r['Counter_Name'], 0) + float(r['Counter_Value'])
for k, v in agg.items():
    if 'nfa' in k:
        print(k, ' '.join(f'{a}={b:.3e}' for a, b in sorted(v.items())))
PY
cat gpurun_out/pmc_lanes.txt

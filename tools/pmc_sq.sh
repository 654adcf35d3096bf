#!/bin/bash
# GPU box: one rocprofv3 --pmc pass (<= 8 SQ counters) over tools/sweep_probe.py; prints per-kernel sums.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc ${COUNTERS:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS} --output-format csv -d $OUT -o p -- python3 -u tools/sweep_probe.py --reps 1 > $OUT/log.txt 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(dict)
for f in glob.glob('gpurun_out/pmc_sq/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0][-40:]
        agg[k][r['Counter_Name']] = agg[k].get(r['Counter_Name'], 0) + float(r['Counter_Value'])
for k, v in agg.items():
    if 'sw_' in k:
        print(k, ' '.join(f'{a}={b:.3e}' for a, b in sorted(v.items())))
PY

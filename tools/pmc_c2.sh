#!/bin/bash
# GPU box: two rocprofv3 --pmc passes (8 SQ counters each) over the C2 bench (LDS bank conflicts,
# VALU utilisation, waits) -> gpurun_out/pmc_c2.json (tools/pmc_summary.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_c2
mkdir -p $OUT
A="SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS"
B="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
C2="--steps 2 --warmup 1 --no-cpu-baseline --latency-batches 0"
timeout -s KILL 150 rocprofv3 --pmc $A --output-format csv -d $OUT/c2_a -o p -- python3 -u bench.py $C2 > $OUT/c2_a.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc $B --output-format csv -d $OUT/c2_b -o p -- python3 -u bench.py $C2 > $OUT/c2_b.log 2>&1 || exit $?
python3 tools/pmc_summary.py $OUT > gpurun_out/pmc_c2.json
python3 - <<'P'
import json
d = json.load(open('gpurun_out/pmc_c2.json'))
for wl, ks in d['workloads'].items():
    for k, v in ks.items():
        if 'sw_' in k:
            print(wl, k, {a: (round(b, 3) if isinstance(b, float) else b) for a, b in v.items() if not a.startswith('SQ_') or a in ('SQ_INSTS_VALU', 'SQ_WAVES', 'SQ_INSTS_LDS')})
P

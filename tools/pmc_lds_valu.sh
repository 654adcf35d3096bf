#!/bin/bash
# GPU box: LDS bank-conflict and VALU-utilisation (divergence) counters for the hot kernels
# (SURVEY.md §8d / north_star), two rocprofv3 --pmc passes (8 SQ counters each) per workload:
#   C2  (sweep: k_sw_count, k_sw_scatter, k_sw_solve)      bench.py default config
#   C3' (general lanes: k_nfa_lanes at 1M keys, HBM arena) bench.py --config 3b, 20M events
# Summary: gpurun_out/pmc_lds_valu.json (tools/pmc_summary.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_lv
mkdir -p $OUT
A="SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS"
B="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
C2="--steps 2 --warmup 1 --no-cpu-baseline --latency-batches 0"
C3="--config 3b --events 20000000 --steps 1 --warmup 0 --no-cpu-baseline --latency-batches 0"
timeout -s KILL 150 rocprofv3 --pmc $A --output-format csv -d $OUT/c2_a -o p -- python3 -u bench.py $C2 > $OUT/c2_a.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc $B --output-format csv -d $OUT/c2_b -o p -- python3 -u bench.py $C2 > $OUT/c2_b.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc $A --output-format csv -d $OUT/c3_a -o p -- python3 -u bench.py $C3 > $OUT/c3_a.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc $B --output-format csv -d $OUT/c3_b -o p -- python3 -u bench.py $C3 > $OUT/c3_b.log 2>&1 || exit $?
python3 tools/pmc_summary.py $OUT > gpurun_out/pmc_lds_valu.json
cat gpurun_out/pmc_lds_valu.json

#!/bin/bash
# GPU box: LDS / VALU / wait counters (two rocprofv3 --pmc passes of 8 SQ counters) and HBM traffic
# (FETCH_SIZE, WRITE_SIZE passes) for one bench config: CFG (bench.py --config, default 2), KEYS
# (recorded in the traffic JSON), BENCH_ARGS.  Summaries: gpurun_out/pmc_<CFG>_lv.json
# (tools/pmc_summary.py) and gpurun_out/pmc_<CFG>_traffic.json (tools/pmc_traffic.py: bench.py --pmc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${CFG:-2}
OUT=gpurun_out/pmc_$CFG
mkdir -p $OUT
A="SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS"
B="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
ARGS="--config $CFG --steps 2 --warmup 1 --no-cpu-baseline --latency-batches 0 --e2e-steps 0 ${BENCH_ARGS}"
if [ -z "$NO_LV" ]; then
  timeout -s KILL 200 rocprofv3 --pmc $A --output-format csv -d $OUT/w_a -o p -- python3 -u bench.py $ARGS > $OUT/w_a.log 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --pmc $B --output-format csv -d $OUT/w_b -o p -- python3 -u bench.py $ARGS > $OUT/w_b.log 2>&1 || exit $?
  python3 tools/pmc_summary.py $OUT > gpurun_out/pmc_${CFG}_lv.json
fi
if [ -z "$NO_TRAFFIC" ]; then
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- python3 -u bench.py $ARGS > $OUT/fetch.log 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- python3 -u bench.py $ARGS > $OUT/write.log 2>&1 || exit $?
  PMC_CONFIG=$CFG PMC_KEYS=${KEYS:-10000} python3 tools/pmc_traffic.py $OUT/fetch $OUT/write > gpurun_out/pmc_${CFG}_traffic.json
fi
[ -z "$NO_LV" ] && cat gpurun_out/pmc_${CFG}_lv.json
true

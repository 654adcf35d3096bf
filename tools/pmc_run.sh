#!/bin/bash
# GPU box: kernel-trace stats + two PMC passes (FETCH_SIZE, WRITE_SIZE) over a short bench run.
# Writes gpurun_out/{stats,pmc_fetch,pmc_write}/ and gpurun_out/pmc.json.
# BENCH_ARGS other than the default C2 run: also set PMC_CONFIG / PMC_KEYS (recorded in pmc.json,
# bench.py uses the traffic only for the same config and key count).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0 --e2e-steps 0 ${BENCH_ARGS}"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats -o run -- python3 -u bench.py $ARGS > gpurun_out/stats.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o p -- python3 -u bench.py $ARGS > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o p -- python3 -u bench.py $ARGS > gpurun_out/pmc_write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc.json
cat gpurun_out/pmc.json

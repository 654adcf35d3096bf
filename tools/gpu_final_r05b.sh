#!/bin/bash
# GPU box, round 5 (staged count-sequence scatter): rocprof kernel stats + PMC HBM traffic for C2, C3', C4,
# C5 on the final library, the traffic files placed where bench.py reads them, then bench lines for C2,
# C3' and C3.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_prof_r05.sh || exit 1
cp gpurun_out/pmc.json profiles/pmc_traffic_c2.json || exit 1
for c in 3b 4 5; do cp gpurun_out/pmc_${c}_traffic.json profiles/pmc_traffic_c$c.json || exit 1; done
mkdir -p gpurun_out/traffic && cp profiles/pmc_traffic_c*.json gpurun_out/traffic/
CONFIGS="c2 c3b c3" bash tools/gpu_bench_all.sh

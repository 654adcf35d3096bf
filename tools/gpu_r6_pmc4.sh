#!/bin/bash
# GPU box: C4 (ordered) PMC traffic on the final library, then the N=8 one-GPU rehearsal
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH_ARGS="--no-expanded" NO_LV=1 CFG=4 KEYS=1000 bash tools/pmc_cfg.sh > gpurun_out/pmc_cfg_4.log 2>&1 || { tail -5 gpurun_out/pmc_cfg_4.log; exit 1; }
cp gpurun_out/pmc_4_traffic.json gpurun_out/pmc_4o_traffic.json
echo "pmc c4 done"
bash tools/gpu_rehearsal_r06.sh | tee gpurun_out/rehearsal_r06.txt

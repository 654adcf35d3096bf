#!/bin/bash
# GPU box: why k_sw_lean costs more at 100k keys (C5) than at 10k (C2).  Phase stamps (stamps build,
# tools/sweep_probe.py) for C2 and C5 at 10k and 100k keys, then plain bench lines (tools/gpu_keys_agg.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export SIDDHI_HIP_DIAG_LIB=siddhi_amd/libsiddhi_hip_stamps.so
for spec in "2 10000" "2 100000" "5 10000 --agg" "5 100000 --agg"; do
  set -- $spec
  timeout -k 10 200 python3 -u tools/sweep_probe.py --config $1 --keys $2 $3 --reps 2 > gpurun_out/lk_$1_$2.log 2>&1 || { tail -20 gpurun_out/lk_$1_$2.log; exit 1; }
  echo "== config $1 keys $2"; tail -8 gpurun_out/lk_$1_$2.log
done
unset SIDDHI_HIP_DIAG_LIB
bash tools/gpu_keys_agg.sh

#!/bin/bash
# GPU box: k_labs_w phase stamps (diagnostic build) on C4, ordered and with 1 % disorder.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in 0.01 0; do
  SIDDHI_HIP_DIAG_LIB=siddhi_amd/libsiddhi_hip_stamps.so timeout -k 10 240 python -u tools/labs_probe.py --disorder $d --reps 2 \
    > gpurun_out/r6_labs_probe_$d.txt 2>&1 || { tail -5 gpurun_out/r6_labs_probe_$d.txt; exit 1; }
  cat gpurun_out/r6_labs_probe_$d.txt
done

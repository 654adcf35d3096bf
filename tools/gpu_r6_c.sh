#!/bin/bash
# GPU box, round 6: labs tests + C4 benches, then the phase probe (diagnostic build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r6_labs.sh || exit $?
SIDDHI_HIP_DIAG_LIB=siddhi_amd/libsiddhi_hip_stamps.so timeout -k 10 240 python -u tools/labs_probe.py --disorder 0.01 --reps 1 \
  > gpurun_out/r6_labs_probe_d.txt 2>&1 || { tail -5 gpurun_out/r6_labs_probe_d.txt; exit 1; }
cat gpurun_out/r6_labs_probe_d.txt

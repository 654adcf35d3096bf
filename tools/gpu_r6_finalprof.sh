#!/bin/bash
# GPU box: round-6 measurement on the final library (tools/gpu_prof_r06.sh), then the N=8 rehearsal
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_prof_r06.sh || exit 1
bash tools/gpu_rehearsal_r06.sh | tee gpurun_out/rehearsal_r06.txt

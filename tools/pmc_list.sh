#!/bin/bash
# GPU box: list the PMC counters rocprofv3 offers on this device (gpurun_out/counters.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1
grep -c . gpurun_out/counters.txt

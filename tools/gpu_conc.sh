#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/conc_probe.py 2>&1 | tee gpurun_out/conc_probe.txt

#!/bin/bash
# GPU box: rocprof kernel stats of C4 with the fused clock and with the device-wide scan (SHP_LABS_SCAN_CLOCK=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--config 4 --steps 3 --warmup 1 --no-cpu-baseline --no-expanded --latency-batches 0 --e2e-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4s_fused -o run -- python3 -u bench.py $Q > gpurun_out/c4s_fused.log 2>&1 || { tail -5 gpurun_out/c4s_fused.log; exit 1; }
export SHP_LABS_SCAN_CLOCK=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4s_scan -o run -- python3 -u bench.py $Q > gpurun_out/c4s_scan.log 2>&1 || { tail -5 gpurun_out/c4s_scan.log; exit 1; }
echo done

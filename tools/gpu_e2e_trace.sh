#!/bin/bash
# GPU box: rocprofv3 kernel + memory-copy trace of the end-to-end ingest (C2, bench.py end_to_end), one form
# per run, and the copy/kernel overlap summary of each (tools/overlap.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in serial pipelined pipelined_narrow; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2e_trace_$m -o run -- \
    python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-expanded --latency-batches 0 --e2e-steps 2 --e2e-modes $m \
    > gpurun_out/e2e_trace_$m.log 2>&1 || { tail -5 gpurun_out/e2e_trace_$m.log; exit 1; }
  python3 tools/overlap.py gpurun_out/e2e_trace_$m $m || { head -c 600 $(ls gpurun_out/e2e_trace_$m/*memory_copy* | head -1); exit 1; }
done

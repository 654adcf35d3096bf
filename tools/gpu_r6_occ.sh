#!/bin/bash
# (SHP_LA_SCAT_LDS, the LDS padding this A/B used, was removed after it: profiles/r06_scatter_occupancy.txt)
# GPU box: C4 multisplit scatter duration against its resident waves (dynamic LDS padded by SHP_LA_SCAT_LDS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--config 4 --steps 3 --warmup 1 --no-cpu-baseline --no-expanded --latency-batches 0 --e2e-steps 0"
for l in 0 16384 24576 32768 40960 53248; do
  export SHP_LA_SCAT_LDS=$l
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/occ_$l -o run -- python3 -u bench.py $Q > gpurun_out/occ_$l.log 2>&1 || { tail -5 gpurun_out/occ_$l.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/occ_$l/run_kernel_stats.csv')):
    if 'k_la_ms_scatter' in r['Name'] or 'k_labs_w<true, false>' in r['Name']: print('lds $l', r['Name'][:40], round(float(r['AverageNs'])/1e3,1), 'us')
"
done

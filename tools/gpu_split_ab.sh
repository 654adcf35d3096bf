#!/bin/bash
# GPU box: k_gs_scatter A/B (in-tree library vs AB_LIB), kernel stats per variant under rocprofv3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in new base; do
  if [ $v = base ]; then export SIDDHI_HIP_DIAG_LIB=$AB_LIB; else unset SIDDHI_HIP_DIAG_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/split_$v -o split -- python3 -u tools/split_probe.py > gpurun_out/split_$v.log 2>&1 || { tail -20 gpurun_out/split_$v.log; exit 1; }
  tail -2 gpurun_out/split_$v.log
  f=$(find gpurun_out/split_$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_gs" in r["Name"] or "sw_scatter" in r["Name"] or "k_sw_lean" in r["Name"]:
        print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e6, 4), "ms")
PY
done

#!/bin/bash
# Build libsiddhi_hip.so from the sources of another git revision, for A/B timing on one box:
#   tools/build_variant.sh <rev> <name>  ->  siddhi_amd/<name>.so
#   SIDDHI_HIP_DIAG_LIB=siddhi_amd/<name>.so python tools/sweep_probe.py
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2
d=$(mktemp -d)
git archive "$rev" siddhi_amd/csrc include | tar -x -C "$d"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared ${EXTRA} -o "siddhi_amd/$name.so" \
  "$d/siddhi_amd/csrc/engine.hip" "$d/siddhi_amd/csrc/synth.hip" "$d/siddhi_amd/csrc/shard.hip" \
  $( [ -f "$d/siddhi_amd/csrc/group.hip" ] && echo "$d/siddhi_amd/csrc/group.hip -lrccl" )
rm -rf "$d"
echo "siddhi_amd/$name.so"

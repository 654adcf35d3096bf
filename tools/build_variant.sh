#!/bin/bash
# Build libsiddhi_hip.so from the sources of another git revision, for A/B timing on one box:
#   tools/build_variant.sh <rev> <name> [extra hipcc flags]  ->  siddhi_amd/<name>.so
#   SIDDHI_HIP_DIAG_LIB=siddhi_amd/<name>.so python bench.py ...
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2; shift 2
d=$(mktemp -d)
git archive "$rev" siddhi_amd/csrc include | tar -x -C "$d"
# the include path of the sources is ../../include relative to csrc: keep the tree's shape
python3 -m siddhi_amd.build --src "$d" --out "$name.so" "$@" > /dev/null
rm -rf "$d"
echo "siddhi_amd/$name.so"

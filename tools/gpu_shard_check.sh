#!/bin/bash
# GPU box: exchange tests, exchange kernel timings (current lib vs SHARD_AB_LIB), and the N=2
# rehearsal of bench.py (both ranks on cuda:0, collectives over gloo).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_shard_device.py -x -v --timeout 120 --timeout-method thread > gpurun_out/shard_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/shard_probe.py > gpurun_out/shard_probe.log 2>&1 || exit $?
if [ -n "$SHARD_AB_LIB" ]; then
  SIDDHI_HIP_DIAG_LIB=$SHARD_AB_LIB timeout -k 10 120 python -u tools/shard_probe.py > gpurun_out/shard_probe_ab.log 2>&1 || exit $?
fi
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --same-device --steps 3 --warmup 1 --events ${REHEARSAL_EVENTS:-20000000} > gpurun_out/same_device.log 2>&1 || exit $?

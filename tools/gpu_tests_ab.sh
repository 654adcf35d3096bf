cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || exit $?
AB_LIB=siddhi_amd/libsiddhi_hip_base.so bash tools/ab_bench.sh

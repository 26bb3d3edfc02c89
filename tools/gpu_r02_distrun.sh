#!/bin/bash
# round 2: the multi-rank program runtime (halo and vertex-cut layouts) and the partitioned
# bench contract on the HIP kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_run.py tests/test_gpu_dist.py -m gpu -v --timeout 240 \
    --timeout-method thread -x > gpurun_out/dr_tests.log 2>&1
rc=$?
tail -n 6 gpurun_out/dr_tests.log
exit $rc

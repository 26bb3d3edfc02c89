#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -v --timeout 240 --timeout-method thread \
    -k "self_launch or rccl_one_rank" > gpurun_out/sl_tests.log 2>&1
rc=$?
tail -n 4 gpurun_out/sl_tests.log
exit $rc

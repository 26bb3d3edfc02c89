#!/bin/bash
# round 2: head-attention kernels + GAT program tests, the GAT e2e epochs, then the R-MAT
# SpMM profile (kernel trace + FETCH_SIZE).  First failing step ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_torch_ext.py tests/test_gpu_dsl.py -x -q \
    --timeout 300 --timeout-method thread -k "head_attn or row_stats or gat" > gpurun_out/r02_attn_tests.log 2>&1 &&
PROGS="gat_products gat_products_h8" ITERS=30 bash tools/gpu_dsl_bench.sh &&
bash tools/gpu_rmat_prof.sh
rc=$?
tail -n 3 gpurun_out/r02_attn_tests.log
cat gpurun_out/dsl_e2e.txt
exit $rc

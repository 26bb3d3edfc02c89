#!/bin/bash
# round 2: GAT row-statistics with parked edge terms: kernel + program tests, op timings,
# e2e GAT epochs and their kernel traces.  First failing step ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_torch_ext.py tests/test_gpu_dsl.py -x -q \
    --timeout 300 --timeout-method thread -k "head_attn or row_stats or gat" > gpurun_out/r02_p_tests.log 2>&1 &&
timeout -k 10 400 python -u tools/gat_bench.py > gpurun_out/r02_gat_bench.jsonl 2> gpurun_out/r02_gat_bench.err &&
PROGS="gat_products gat_products_h8" ITERS=30 bash tools/gpu_dsl_bench.sh &&
PROGS="gat_products gat_products_h8 gcn_products" bash tools/gpu_r02_e2e_prof.sh
rc=$?
tail -n 3 gpurun_out/r02_p_tests.log
grep stats gpurun_out/r02_gat_bench.jsonl
cat gpurun_out/dsl_e2e.txt
exit $rc

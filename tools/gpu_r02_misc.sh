#!/bin/bash
# round 2: the 64-bit address test, the GAT DSL programs vs the float64 IR executor, the
# e2e GAT epochs (1 and 8 heads), then the GAT PMC passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r02_large_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_dsl.py -x -q --timeout 300 --timeout-method thread -k "gat" \
    > gpurun_out/r02_dsl_gat_tests.log 2>&1 &&
PROGS="gat_products gat_products_h8" ITERS=30 bash tools/gpu_dsl_bench.sh &&
bash tools/gpu_pmc_gat.sh
rc=$?
tail -n 4 gpurun_out/r02_large_tests.log gpurun_out/r02_dsl_gat_tests.log
cat gpurun_out/dsl_e2e.txt
exit $rc

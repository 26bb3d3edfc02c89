#!/bin/bash
# round 2: the GAT row-statistics path -- kernel parity tests, the mirror / DSL GAT tests,
# then the op timings.  First failing step ends it.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 240 --timeout-method thread \
    -k "row_stats or gat_bwd_fused_recompute" > gpurun_out/r02_stats_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_torch_ext.py tests/test_gpu_dsl.py -x -q --timeout 300 \
    --timeout-method thread -k "gat" > gpurun_out/r02_stats_gat_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/gat_bench.py > gpurun_out/r02_gat_bench.jsonl 2> gpurun_out/r02_gat_bench.err
rc=$?
tail -n 5 gpurun_out/r02_stats_tests.log gpurun_out/r02_stats_gat_tests.log
cat gpurun_out/r02_gat_bench.jsonl
exit $rc

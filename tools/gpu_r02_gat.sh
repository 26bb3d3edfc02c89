#!/bin/bash
# round-2 GAT work: kernel parity tests for the GAT / SpMM paths, the torch mirror tests,
# then op timings on the Products shape.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    -k "gat or spmm or softmax" > gpurun_out/r02_gat_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_torch_ext.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r02_torch_ext_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_dsl.py -x -q --timeout 300 --timeout-method thread -k "gat" > gpurun_out/r02_dsl_gat_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/gat_bench.py > gpurun_out/r02_gat_bench.jsonl 2> gpurun_out/r02_gat_bench.err
rc=$?
tail -n 3 gpurun_out/r02_gat_tests.log gpurun_out/r02_torch_ext_tests.log gpurun_out/r02_dsl_gat_tests.log
cat gpurun_out/r02_gat_bench.jsonl
exit $rc

#!/bin/bash
# GAT / SpMM kernel parity tests, the distributed-layout GPU tests, op timings, PMC passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_large.py -x -q --timeout 240 \
    --timeout-method thread -k "gat or spmm or softmax or 2pow31 or refused" > gpurun_out/r02_gat_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_dist_run.py -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/r02_dist_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/gat_bench.py > gpurun_out/r02_gat_bench.jsonl 2> gpurun_out/r02_gat_bench.err &&
bash tools/gpu_pmc_gat.sh
rc=$?
tail -n 3 gpurun_out/r02_gat_tests.log gpurun_out/r02_dist_tests.log
cat gpurun_out/r02_gat_bench.jsonl
exit $rc

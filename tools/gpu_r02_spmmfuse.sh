#!/bin/bash
# SpMM rows + hub chunks in one launch: parity (kernel tests + fuzz) and the R-MAT bench field
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dist.py -m gpu -q -x --timeout 120 \
    --timeout-method thread > gpurun_out/sf_tests.log 2>&1 &&
GALA_FUZZ_CASES=400 timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q -x --timeout 300 \
    --timeout-method thread > gpurun_out/sf_fuzz.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-gat > gpurun_out/sf_bench.json 2> gpurun_out/sf_bench.err
rc=$?
tail -n 2 gpurun_out/sf_tests.log gpurun_out/sf_fuzz.log
python3 -c "import json; d=json.load(open('gpurun_out/sf_bench.json')); print(d['roofline']['kernel_ms'], d['rmat'])"
exit $rc

#!/bin/bash
# GPU: kernel + mirror parity tests, then the GAT config timings.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_torch_ext.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_edge.log 2>&1; rc=$?; echo pytest=$rc; tail -3 gpurun_out/pytest_edge.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/configs_bench.py --which ${WHICH:-gat} > gpurun_out/configs.jsonl 2> gpurun_out/configs.err; echo configs=$?
cat gpurun_out/configs.jsonl

#!/bin/bash
# GAT rows + hub chunks in one grid: parity (kernel tests, dist tests, fuzz) on the new
# library, then old / new A/B of the 8-head and 1-head statistics pair on R-MAT and uniform
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dist.py tests/test_gpu_torch_ext.py -m gpu \
    -q -x --timeout 120 --timeout-method thread > gpurun_out/gf_tests.log 2>&1 &&
GALA_FUZZ_CASES=400 timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q -x --timeout 300 \
    --timeout-method thread > gpurun_out/gf_fuzz.log 2>&1 || { tail -5 gpurun_out/gf_tests.log gpurun_out/gf_fuzz.log; exit 1; }
rm -f gpurun_out/gatv_ref_*.pt gpurun_out/gat_variants.jsonl
for g in rmat uniform; do
  rm -f gpurun_out/gatv_ref_*.pt
  for v in old new; do
    GALA_GRAPH=$g timeout -k 10 150 python -u tools/gat_variants.py abx/$v >> gpurun_out/gat_variants.jsonl 2>> gpurun_out/gat_variants.err || exit $?
  done
done
tail -n 2 gpurun_out/gf_tests.log gpurun_out/gf_fuzz.log
cat gpurun_out/gat_variants.jsonl

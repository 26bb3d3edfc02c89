#!/bin/bash
# round 2 end: e2e epochs of the config programs on HEAD and a 4000-case randomised sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PROGS="gcn_products gat_products gat_products_h8 gcn_arxiv sage_reddit_sampled gcn3_papers10" ITERS=50 \
    bash tools/gpu_dsl_bench.sh || exit $?
GALA_FUZZ_CASES=2000 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q -x --timeout 500 \
    --timeout-method thread > gpurun_out/e2ef_fuzz.log 2>&1
rc=$?
cat gpurun_out/dsl_e2e.txt
tail -n 2 gpurun_out/e2ef_fuzz.log
exit $rc

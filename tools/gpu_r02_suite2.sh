#!/bin/bash
# round 2: the whole -m gpu suite + smoke (log kept for profiles/), then the GAT e2e epochs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 960 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread \
    > gpurun_out/r02_gpu_tests.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02_smoke.log 2>&1 &&
PROGS="gat_products gat_products_h8" ITERS=30 bash tools/gpu_dsl_bench.sh
rc=$?
tail -n 3 gpurun_out/r02_gpu_tests.log gpurun_out/r02_smoke.log
cat gpurun_out/dsl_e2e.txt
exit $rc

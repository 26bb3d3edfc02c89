#!/bin/bash
# round 2: the whole -m gpu suite, smoke(), and the GAT op timings (one box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 960 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread \
    > gpurun_out/r02_gpu_tests.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02_smoke.log 2>&1 &&
timeout -k 10 300 python -u tools/gat_bench.py > gpurun_out/r02_gat_bench.jsonl 2> gpurun_out/r02_gat_bench.err
rc=$?
tail -n 3 gpurun_out/r02_gpu_tests.log gpurun_out/r02_smoke.log
cat gpurun_out/r02_gat_bench.jsonl
exit $rc

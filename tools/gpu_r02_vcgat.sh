#!/bin/bash
# round 2: the vertex-cut GAT training pair (simulated-rank HIP tests, the partitioned bench
# path over RCCL at world 1) and the full-scale partitioned bench line with its GAT field
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/vc_dist_tests.log 2>&1 &&
GALA_BENCH_DIST=1 timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline \
    > gpurun_out/vc_bench_dist1.json 2> gpurun_out/vc_bench_dist1.err
rc=$?
tail -n 4 gpurun_out/vc_dist_tests.log
cat gpurun_out/vc_bench_dist1.json
exit $rc

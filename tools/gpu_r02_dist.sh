#!/bin/bash
# round-2 multi-GPU plumbing on one GPU: simulated-rank HIP tests, the N=1 bench line,
# and the 2-rank gloo rehearsal of the self-launching strong-scaling bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/r02_dist_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r02_bench1.json 2> gpurun_out/r02_bench1.err &&
GALA_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --scale 0.1 --steps 5 --warmup 2 \
    > gpurun_out/r02_bench2_gloo.json 2> gpurun_out/r02_bench2_gloo.err
rc=$?
tail -3 gpurun_out/r02_dist_tests.log
exit $rc

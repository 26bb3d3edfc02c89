#!/bin/bash
# round 2, session 3: the whole -m gpu suite, smoke(), the N=1 bench line, the one-rank
# RCCL contract run of the partitioned path, and the 2-rank gloo rehearsal (one box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread \
    > gpurun_out/s3_gpu_tests.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/s3_bench1.json 2> gpurun_out/s3_bench1.err &&
GALA_BENCH_DIST=1 timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/s3_bench_dist1.json 2> gpurun_out/s3_bench_dist1.err &&
GALA_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --scale 0.1 --steps 5 --warmup 2 \
    > gpurun_out/s3_bench2_gloo.json 2> gpurun_out/s3_bench2_gloo.err
rc=$?
tail -n 3 gpurun_out/s3_gpu_tests.log gpurun_out/s3_smoke.log
cat gpurun_out/s3_bench1.json gpurun_out/s3_bench_dist1.json gpurun_out/s3_bench2_gloo.json
exit $rc

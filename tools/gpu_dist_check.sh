#!/bin/bash
# GPU tests + single-GPU bench; then a 1-GPU rehearsal of the multi-rank launch path
# (torchrun with nproc 1 exercises init/barrier/all-reduce of bench.py).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "STOP rc=$1"; return 1;; esac; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest=$rc; ok $rc || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc=$?; echo bench=$rc; ok $rc || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_trun.json 2> gpurun_out/bench_trun.err; echo trun=$?
# 2 ranks sharing the one GPU over gloo (rehearsal of the N>1 code path; not a perf number)
GALA_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 3 --warmup 1 --scale 0.25 --no-cpu-baseline > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err; echo gloo2=$?

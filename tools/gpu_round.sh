#!/bin/bash
# GPU: the whole -m gpu suite, the galac end-to-end config programs, and a rocprofv3
# kernel-trace of one of them ($PROF_PROG, default gcn_products).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest=$rc
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/gpu_dsl_bench.sh || exit $?
P=${PROF_PROG:-gcn_products}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_e2e -o $P -- \
    $GRAFT_REPO_ROOT/gala-gnn-acceleration-language_amd/progs/$P/gala_prog --synthetic --iters 20 \
    > $GRAFT_REPO_ROOT/gpurun_out/prof_e2e.log 2>&1; echo prof=$?

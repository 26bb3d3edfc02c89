#!/bin/bash
# GPU: the galac-generated programs (tests/test_gpu_dsl.py) + optional $EXTRA
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 gala-gnn-acceleration-language_amd/progs/gat/gala_prog --synthetic --iters 3 > gpurun_out/gat_prog.log 2>&1; rc=$?; echo gat_prog=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests/test_gpu_dsl.py -m gpu -q -x > gpurun_out/pytest_dsl.log 2>&1; rc=$?; echo pytest=$rc
case $rc in 0|1) ;; *) exit $rc;; esac
if [ -n "$EXTRA" ]; then bash -c "$EXTRA"; echo extra=$?; fi

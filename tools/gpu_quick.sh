#!/bin/bash
# GPU tests (+ optional extra command in $EXTRA)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest=$rc
case $rc in 0|1) ;; *) exit $rc;; esac
if [ -n "$EXTRA" ]; then bash -c "$EXTRA"; echo extra=$?; fi

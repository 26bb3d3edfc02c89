#!/bin/bash
# smoke + GPU parity tests + short bench (+ sweep).  Each GPU step has its own limit;
# a crash/timeout stops the script.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "STOP rc=$1"; return 1;; esac; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke=$rc; ok $rc || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest=$rc; ok $rc || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc=$?; echo bench=$rc; ok $rc || exit $rc
if [ -n "$SWEEP" ]; then
timeout -k 10 300 python tools/spmm_sweep.py $SWEEP > gpurun_out/sweep.log 2> gpurun_out/sweep.err; echo sweep=$?
fi

#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "STOP rc=$1"; return 1;; esac; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke=$rc; ok $rc || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest=$rc; ok $rc || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc=$?; echo bench=$rc; ok $rc || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof1.log" 2>&1; echo prof=$?
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/spmm_sweep.py > gpurun_out/sweep.log 2> gpurun_out/sweep.err; echo sweep=$?

#!/bin/bash
# round 2 end: the whole -m gpu suite and smoke() on HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread \
    > gpurun_out/end_gpu_tests.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/end_smoke.log 2>&1
rc=$?
tail -n 2 gpurun_out/end_gpu_tests.log gpurun_out/end_smoke.log
exit $rc

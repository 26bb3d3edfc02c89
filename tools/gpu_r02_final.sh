#!/bin/bash
# round 2 record run: the whole -m gpu suite, smoke(), a larger randomised sweep, the N=1
# bench line, and rocprofv3 kernel stats of the bench without the R-MAT family (so the SpMM
# average is the headline graph's alone).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread \
    > gpurun_out/fin_gpu_tests.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 &&
GALA_FUZZ_CASES=${FUZZ:-1000} timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q -x --timeout 300 \
    --timeout-method thread > gpurun_out/fin_fuzz.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/fin_bench1.json 2> gpurun_out/fin_bench1.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fin_prof -o run \
    -- python3 $R/bench.py --no-rmat --no-cpu-baseline > $R/gpurun_out/fin_prof_bench.json 2> $R/gpurun_out/fin_prof_bench.err
rc=$?
cd $R
tail -n 2 gpurun_out/fin_gpu_tests.log gpurun_out/fin_smoke.log gpurun_out/fin_fuzz.log
cat gpurun_out/fin_bench1.json
exit $rc

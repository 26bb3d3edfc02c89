#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_rmat -o run -- \
    python3 $R/tools/rmat_prof.py > $R/gpurun_out/prof_rmat.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/prof_rmat_fetch -o run -- \
    python3 $R/tools/rmat_prof.py > $R/gpurun_out/prof_rmat_fetch.log 2>&1 || exit $?
cat $R/gpurun_out/prof_rmat.log | grep -v amdgpu.ids
head -12 $R/gpurun_out/prof_rmat/run_kernel_stats.csv | cut -c1-170

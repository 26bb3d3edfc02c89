#!/bin/bash
# round 2: the N=1 bench line (GCN headline + R-MAT + the config-3 GAT layer) and the
# rocprofv3 kernel-trace stats of the same command (one box).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u bench.py > gpurun_out/bp_bench1.json 2> gpurun_out/bp_bench1.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bp_prof -o run \
    -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bp_prof_bench.json 2> $R/gpurun_out/bp_prof_bench.err
rc=$?
cat $R/gpurun_out/bp_bench1.json
exit $rc

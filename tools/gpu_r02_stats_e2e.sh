#!/bin/bash
# round 2: e2e GAT epochs with the row-statistics backward (default) and without it
# (GALA_GAT_ROWSTATS=0), plus a kernel trace of the 8-head program.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
PROGS="gat_products gat_products_h8" ITERS=30 bash tools/gpu_dsl_bench.sh || exit $?
cp gpurun_out/dsl_e2e.txt gpurun_out/dsl_e2e_rowstats.txt
GALA_GAT_ROWSTATS=0 PROGS="gat_products gat_products_h8" ITERS=30 bash tools/gpu_dsl_bench.sh || exit $?
cp gpurun_out/dsl_e2e.txt gpurun_out/dsl_e2e_norowstats.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_e2e_h8 -o run -- \
    $R/gala-gnn-acceleration-language_amd/progs/gat_products_h8/gala_prog --synthetic --iters 10 \
    > $R/gpurun_out/prof_e2e_h8.log 2>&1 || exit $?
cat $R/gpurun_out/dsl_e2e_rowstats.txt $R/gpurun_out/dsl_e2e_norowstats.txt
head -12 $R/gpurun_out/prof_e2e_h8/run_kernel_stats.csv | cut -c1-150

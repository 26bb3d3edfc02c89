#!/bin/bash
# round 2: end-to-end epochs of the config programs (galac-generated), a kernel trace of
# the 8-head GAT program, and the GAT PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
PROGS="gcn_products gat_products gat_products_h8 gcn_arxiv sage_reddit_sampled gcn3_papers10" ITERS=50 \
    bash tools/gpu_dsl_bench.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_e2e_h8 -o run -- \
    $R/gala-gnn-acceleration-language_amd/progs/gat_products_h8/gala_prog --synthetic --iters 10 \
    > $R/gpurun_out/prof_e2e_h8.log 2>&1 || exit $?
bash $R/tools/gpu_pmc_gat.sh || exit $?
cat $R/gpurun_out/dsl_e2e.txt

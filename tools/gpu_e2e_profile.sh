#!/bin/bash
# GPU: rocprofv3 kernel-trace stats of the galac-generated e2e programs (synthetic datasets
# of the configs' shapes, 20 epochs each); one directory per program under gpurun_out/.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for p in ${PROGS:-gat_products gcn_products gcn3_papers10 sage_reddit_sampled}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/e2e_$p -o run -- $R/gala-gnn-acceleration-language_amd/progs/$p/gala_prog --synthetic --iters 20 > $R/gpurun_out/e2e_$p.log 2>&1 || exit $?
done

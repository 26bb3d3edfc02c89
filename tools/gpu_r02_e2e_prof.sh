#!/bin/bash
# kernel traces of the config programs' epochs (galac-generated, synthetic datasets)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for p in ${PROGS:-gat_products gat_products_h8 gcn_products}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_e2e_$p -o run -- \
        $R/gala-gnn-acceleration-language_amd/progs/$p/gala_prog --synthetic --iters 10 \
        > $R/gpurun_out/prof_e2e_$p.log 2>&1 || exit $?
done
echo done

#!/bin/bash
# GPU: end-to-end training runs of the bench/dsl programs (galac-generated) on synthetic
# datasets of the configs' shapes.  Each line of gpurun_out/dsl_e2e.txt: program, the
# program's own summary line, then its result line "fwd_mean_s,epoch_mean_s".
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/dsl_e2e.txt
: > $out
for p in ${PROGS:-gcn_products gcn_products_inference gat_products gat_products_h8 gcn_arxiv sage_reddit_sampled gcn3_papers10}; do
    exe=gala-gnn-acceleration-language_amd/progs/$p/gala_prog
    timeout -k 10 300 $exe --synthetic --iters ${ITERS:-100} > gpurun_out/dsl_$p.log 2>&1; rc=$?
    echo "$p rc=$rc $(head -1 gpurun_out/dsl_$p.log) | $(tail -1 gpurun_out/dsl_$p.log)" >> $out
    echo "$p rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done

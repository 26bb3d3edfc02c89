#!/bin/bash
# GAT forward kernel variants (exp/<name>/libgala_hip.so), one process each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/gatv_ref_*.pt
for v in ${VARIANTS:-base pf dpp nomask pfdpp pfdpp4 all all4}; do
  timeout -k 10 120 python -u tools/gat_variants.py exp/$v >> gpurun_out/gat_variants.jsonl 2>> gpurun_out/gat_variants.err || exit $?
done
cat gpurun_out/gat_variants.jsonl

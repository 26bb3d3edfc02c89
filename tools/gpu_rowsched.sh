#!/bin/bash
# GPU: kernel tests, then SpMM timings on uniform and R-MAT Products-shaped graphs
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_torch_ext.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1; rc=$?; echo pytest=$rc; tail -2 gpurun_out/pytest_k.log
[ $rc -eq 0 ] || exit $rc
for g in uniform rmat; do
timeout -k 10 300 python tools/spmm_sweep.py --graph $g --F 8,16,32,64,128,256 --ops spmm,sddmm,gat,sddvv,softmax > gpurun_out/sw_$g.jsonl 2>/dev/null || exit 1
echo "$g $(python -c "import json;print(' '.join('%s/F%s=%.3f'%(d['op'],d.get('F','-'),d['ms']) for d in map(json.loads,open('gpurun_out/sw_$g.jsonl'))))")"
done

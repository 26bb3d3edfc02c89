#!/bin/bash
# round 2: 2-rank rehearsal of the self-launching strong-scaling bench on one GPU over gloo
# (every layout candidate and the vertex-cut GAT field; not a performance number)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
GALA_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --scale 0.1 --steps 4 --warmup 1 \
    > gpurun_out/g2_bench.json 2> gpurun_out/g2_bench.err
rc=$?
grep '^{' gpurun_out/g2_bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['comm']['mode'], d['gat'])"
exit $rc

#!/bin/bash
# bench contract on the GPU: stdout holds exactly one JSON line, N=1 and the one-rank RCCL
# partitioned path
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bc_n1.json 2> gpurun_out/bc_n1.err &&
GALA_BENCH_DIST=1 timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline \
    > gpurun_out/bc_dist1.json 2> gpurun_out/bc_dist1.err
rc=$?
wc -l gpurun_out/bc_n1.json gpurun_out/bc_dist1.json
python3 -c "import json; [print(f, json.load(open(f))['value']) for f in ('gpurun_out/bc_n1.json', 'gpurun_out/bc_dist1.json')]"
exit $rc

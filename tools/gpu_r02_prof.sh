#!/bin/bash
# round 2 profile refresh: the bench line, rocprofv3 kernel-trace stats of bench.py, the
# PMC FETCH_SIZE / WRITE_SIZE passes (separate runs; the uniform headline only, so the
# per-kernel averages are not mixed with the R-MAT family's launches), and the 2-rank gloo
# rehearsal of the self-launching strong-scaling bench.  First failing step ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
OUT="$R/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 400 python -u bench.py > "$OUT/r02_bench.json" 2> "$OUT/r02_bench.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_stats" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-rmat > "$OUT/prof_stats.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/prof_fetch" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-rmat > "$OUT/prof_fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/prof_write" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-rmat > "$OUT/prof_write.log" 2>&1 || exit $?
python3 "$R/tools/pmc_traffic.py" "$OUT/prof_fetch" "$OUT/prof_write" "$OUT/traffic.json" > "$OUT/traffic.log" 2>&1
cd "$R"
GALA_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --scale 0.25 --steps 5 --warmup 2 \
    > "$OUT/r02_bench2_gloo.json" 2> "$OUT/r02_bench2_gloo.err" || exit $?
timeout -k 10 300 python -u tools/rmat_sweep.py > "$OUT/r02_rmat_sweep.jsonl" 2> "$OUT/r02_rmat_sweep.err" || exit $?
cat "$OUT/r02_bench.json" "$OUT/traffic.log" "$OUT/r02_rmat_sweep.jsonl"
echo prof_done

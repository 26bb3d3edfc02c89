#!/bin/bash
# Round profile refresh: bench line, rocprofv3 kernel-trace stats of bench.py, PMC
# FETCH_SIZE / WRITE_SIZE passes (separate runs), per-config timings, a kernel trace of the
# GAT config, and the random-gather ceiling.  Every GPU step has its own time limit; the
# first failing step ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
R=$GRAFT_REPO_ROOT
step() { echo "== $1"; }
step bench && timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
cd /tmp && export TMPDIR=/tmp
step stats && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_stats" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_stats.log" 2>&1 || exit $?
step fetch && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/prof_fetch" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/prof_fetch.log" 2>&1 || exit $?
step write && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/prof_write" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/prof_write.log" 2>&1 || exit $?
python3 "$R/tools/pmc_traffic.py" "$OUT/prof_fetch" "$OUT/prof_write" "$OUT/traffic.json" > "$OUT/traffic.log" 2>&1
cd "$R"
step configs && timeout -k 10 600 python tools/configs_bench.py > "$OUT/configs.jsonl" 2> "$OUT/configs.err" || exit $?
cd /tmp
step gatprof && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_gat" -o run -- python3 "$R/tools/configs_bench.py" --which gat > "$OUT/prof_gat.log" 2>&1 || exit $?
cd "$R"
step ceiling && timeout -k 10 60 tools/gather_ceiling > "$OUT/gc32.jsonl" && timeout -k 10 60 tools/gather_ceiling 2449029 126167309 256 > "$OUT/gc256.jsonl" && timeout -k 10 60 tools/gather_ceiling 169343 1335586 128 > "$OUT/gc128.jsonl" || exit $?
echo profile_round_done

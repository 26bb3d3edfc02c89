#!/bin/bash
# rocprofv3: kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE PMC passes of bench.py
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_stats" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_stats.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/prof_fetch" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/prof_fetch.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/prof_write" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/prof_write.log" 2>&1 || exit $?
python3 "$GRAFT_REPO_ROOT/tools/pmc_traffic.py" "$OUT/prof_fetch" "$OUT/prof_write" "$OUT/traffic.json" > "$OUT/traffic.log" 2>&1
echo profile_done
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/spmm_sweep.py --F 32,128 --ops rocsparse,spmm > gpurun_out/sweep_rocsparse.log 2>&1; echo sweep=$?

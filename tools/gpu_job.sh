#!/bin/bash
# Parameterised GPU job for `gpurun`: each argument is one step, run in order; the job
# stops at the first step that fails (and never starts another GPU step after a fault,
# abort or time limit).  Output goes to gpurun_out/.
#
#   tests            python -m pytest tests -m gpu            -> gpurun_out/pytest_gpu.log
#   tests=EXPR       ... -k EXPR ("_or_" stands for " or ")
#   smoke            __graft_entry__.smoke()                -> gpurun_out/smoke.log
#   bench            python bench.py (N = 1 defaults)        -> gpurun_out/bench.json (+ .log)
#   bench=ARGS       python bench.py ARGS (spaces as commas)
#   benchdist        GALA_BENCH_DIST=1 bench.py: the strong-scaling path over RCCL at world 1
#                                                            -> gpurun_out/bench_dist.json
#   prof             rocprofv3 --kernel-trace --stats of bench.py -> gpurun_out/prof_stats/
#   pmc              FETCH_SIZE and WRITE_SIZE passes (one --pmc run each) of bench.py, then
#                    tools/pmc_traffic.py                   -> gpurun_out/traffic.json
#   py=SCRIPT,ARGS   python SCRIPT ARGS                      -> gpurun_out/<script>.log
#   sh=CMD           a preparation command, no GPU (commas as spaces)
#   bin=TAG,CMD      a GPU program (commas as spaces)        -> gpurun_out/TAG.log
#   env=NAME=VALUE   export a variable for the following steps
#   profcmd=TAG,CMD  rocprofv3 --kernel-trace --stats of CMD (commas as spaces; the program
#                    itself right after --)                  -> gpurun_out/prof_TAG/
#   pmccmd=TAG,CMD   FETCH_SIZE / WRITE_SIZE passes of CMD  -> gpurun_out/traffic_TAG.json
#
# e.g. gpurun --timeout 900 -- 'bash tools/gpu_job.sh tests=gat bench prof'
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
export PYTHONPATH="$GRAFT_REPO_ROOT/gala-gnn-acceleration-language_amd${PYTHONPATH:+:$PYTHONPATH}"
BENCH_PROF_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-banded --no-rmat"
# the banded and R-MAT families' SpMMs run the uniform one's row kernel: rocprof and PMC runs
# of bench.py leave them out, so a kernel's average / bytes are the headline graph's (the
# families' own: pmccmd=banded,python3,<repo>/tools/banded_spmm.py,banded and
# pmccmd=rmat,python3,<repo>/tools/rmat_prof.py, merged into profiles/traffic.json under a
# "banded|" / "rmat|" prefix by tools/merge_traffic.py)
BENCH_PMC_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-banded --no-rmat"

step() {  # name, limit, command...
    local name=$1 lim=$2
    shift 2
    echo "[gpu_job] $name: $*" >&2
    timeout -k 10 "$lim" "$@"
    local rc=$?
    echo "[gpu_job] $name rc=$rc" >&2
    return $rc
}

for s in "$@"; do
    case "$s" in
    tests)
        step tests 900 python -u -m pytest tests -m gpu -q -rs -x --timeout 120 --timeout-method thread \
            > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
        tail -3 "$OUT/pytest_gpu.log" ;;
    tests=*)
        k="${s#tests=}"
        step tests 900 python -u -m pytest tests -m gpu -q -rs -x --timeout 120 --timeout-method thread -k "${k//_or_/ or }" \
            > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
        tail -3 "$OUT/pytest_gpu.log" ;;
    smoke)
        step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
            || { tail -30 "$OUT/smoke.log"; exit 1; }
        tail -1 "$OUT/smoke.log" ;;
    bench)
        step bench 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log" || { tail -30 "$OUT/bench.log"; exit 1; }
        cat "$OUT/bench.json" ;;
    bench=*)
        a="${s#bench=}"
        step bench 900 python -u bench.py ${a//,/ } > "$OUT/bench.json" 2> "$OUT/bench.log" || { tail -30 "$OUT/bench.log"; exit 1; }
        cat "$OUT/bench.json" ;;
    benchdist)
        # the partitioned path on this one GPU (RCCL at world 1: the collectives run)
        GALA_BENCH_DIST=1 step benchdist 900 python -u bench.py --no-cpu-baseline > "$OUT/bench_dist.json" \
            2> "$OUT/bench_dist.log" || { tail -30 "$OUT/bench_dist.log"; exit 1; }
        cat "$OUT/bench_dist.json" ;;
    prof)
        (cd /tmp && step prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_stats" -o run \
            -- python3 "$GRAFT_REPO_ROOT/bench.py" $BENCH_PROF_ARGS > "$OUT/prof_stats.log" 2>&1) || exit 1 ;;
    pmc)
        (cd /tmp && step fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/prof_fetch" -o run \
            -- python3 "$GRAFT_REPO_ROOT/bench.py" $BENCH_PMC_ARGS > "$OUT/prof_fetch.log" 2>&1) || exit 1
        (cd /tmp && step write 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/prof_write" -o run \
            -- python3 "$GRAFT_REPO_ROOT/bench.py" $BENCH_PMC_ARGS > "$OUT/prof_write.log" 2>&1) || exit 1
        python3 tools/pmc_traffic.py "$OUT/prof_fetch" "$OUT/prof_write" "$OUT/traffic.json" > "$OUT/traffic.log" 2>&1 ;;
    profcmd=*)
        # profcmd=TAG,prog,args...: rocprofv3 kernel-trace stats of any command (commas = spaces)
        a="${s#profcmd=}"
        tag="${a%%,*}"
        rest="${a#*,}"
        (cd /tmp && step "prof_$tag" 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$tag" -o run \
            -- ${rest//,/ } > "$OUT/prof_$tag.log" 2>&1) || { tail -20 "$OUT/prof_$tag.log"; exit 1; } ;;
    pmccmd=*)
        # pmccmd=TAG,prog,args...: the FETCH_SIZE and WRITE_SIZE passes (one --pmc run each) of
        # any command, then tools/pmc_traffic.py           -> gpurun_out/traffic_TAG.json
        a="${s#pmccmd=}"
        tag="${a%%,*}"
        rest="${a#*,}"
        (cd /tmp && step "fetch_$tag" 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
            -d "$OUT/pmc_${tag}_fetch" -o run -- ${rest//,/ } > "$OUT/pmc_${tag}_fetch.log" 2>&1) || exit 1
        (cd /tmp && step "write_$tag" 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv \
            -d "$OUT/pmc_${tag}_write" -o run -- ${rest//,/ } > "$OUT/pmc_${tag}_write.log" 2>&1) || exit 1
        python3 tools/pmc_traffic.py "$OUT/pmc_${tag}_fetch" "$OUT/pmc_${tag}_write" "$OUT/traffic_$tag.json" \
            > "$OUT/traffic_$tag.log" 2>&1 ;;
    bin=*)
        # bin=TAG,prog,args...: a GPU program (commas = spaces)  -> gpurun_out/TAG.log
        a="${s#bin=}"
        tag="${a%%,*}"
        rest="${a#*,}"
        step "$tag" 300 ${rest//,/ } > "$OUT/$tag.log" 2>&1 || { tail -20 "$OUT/$tag.log"; exit 1; }
        tail -5 "$OUT/$tag.log" ;;
    env=*)
        # env=NAME=VALUE: exported for the steps after it
        export "${s#env=}" ;;
    sh=*)
        # sh=CMD: a host-side preparation command (commas = spaces), e.g. galac
        a="${s#sh=}"
        step sh 300 ${a//,/ } || exit 1 ;;
    py=*)
        a="${s#py=}"
        scr="${a%%,*}"
        rest=""
        [ "$a" != "$scr" ] && rest="${a#*,}"
        step "$scr" 900 python -u $scr ${rest//,/ } > "$OUT/$(basename "$scr" .py).log" 2>&1 \
            || { tail -30 "$OUT/$(basename "$scr" .py).log"; exit 1; }
        tail -5 "$OUT/$(basename "$scr" .py).log" ;;
    *)
        echo "[gpu_job] unknown step $s"; exit 2 ;;
    esac
done
echo "[gpu_job] done"

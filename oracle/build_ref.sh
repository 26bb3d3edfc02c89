#!/usr/bin/env bash
# Compiles the reference's own CPU code (header-only C++, read in place from
# $REF_ROOT, default /root/reference) through oracle/ref_harness.cpp into
# oracle/_ref/libgala_ref.so.  Test infrastructure only; the output directory is
# git-ignored and the reference sources are never copied into this repository.
# Flags follow the reference build (-O3 -fopenmp) with -march=x86-64-v3 instead of
# -march=native so the prebuilt library also runs on the GPU box host CPU.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REF_ROOT="${REF_ROOT:-/root/reference}"
if [ ! -f "$REF_ROOT/src/ops/aggregators.h" ]; then
    echo "reference not present at $REF_ROOT; skipping oracle/_ref build" >&2
    exit 0
fi
TORCH_DIR="$(python3 -c 'import os,torch;print(os.path.dirname(torch.__file__))')"
mkdir -p "$HERE/_ref"
g++ -O3 -march=x86-64-v3 -fopenmp -fPIC -shared -std=c++17 -w \
    -I"$REF_ROOT" \
    -I"$TORCH_DIR/include" -I"$TORCH_DIR/include/torch/csrc/api/include" \
    "$HERE/ref_harness.cpp" -o "$HERE/_ref/libgala_ref.so" \
    -L"$TORCH_DIR/lib" -Wl,-rpath,"$TORCH_DIR/lib" -ltorch_cpu -lc10
echo "built $HERE/_ref/libgala_ref.so"

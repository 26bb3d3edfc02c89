#!/usr/bin/env bash
# Compiles the reference's own CPU code (header-only C++, read in place from
# $REF_ROOT, default /root/reference) through oracle/ref_harness.cpp into
# oracle/_ref/libgala_ref.so.  Test infrastructure only; the output directory is
# git-ignored and the reference sources are never copied into this repository.
#
# Flags follow the reference build (-O3 -fopenmp -march=native, CMakeLists.txt:262-282).
# The library is built here and run on the GPU box's host CPU, so "native" is pinned to
# the ISA both hosts share: x86-64-v4 (AVX-512 F/BW/CD/DQ/VL; this container's Xeon and
# the box's EPYC 9575F both have it).  REF_MARCH / REF_OUT override the ISA and the output
# path (tools/cpu_baseline_flags.py builds variants into /tmp to compare them).
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REF_ROOT="${REF_ROOT:-/root/reference}"
REF_MARCH="${REF_MARCH:-x86-64-v4}"
REF_OUT="${REF_OUT:-$HERE/_ref/libgala_ref.so}"
if [ ! -f "$REF_ROOT/src/ops/aggregators.h" ]; then
    echo "reference not present at $REF_ROOT; skipping oracle/_ref build" >&2
    exit 0
fi
TORCH_DIR="$(python3 -c 'import os,torch;print(os.path.dirname(torch.__file__))')"
mkdir -p "$(dirname "$REF_OUT")"
g++ -O3 -march="$REF_MARCH" -fopenmp -fPIC -shared -std=c++17 -w \
    -I"$REF_ROOT" \
    -I"$TORCH_DIR/include" -I"$TORCH_DIR/include/torch/csrc/api/include" \
    "$HERE/ref_harness.cpp" -o "$REF_OUT" \
    -L"$TORCH_DIR/lib" -Wl,-rpath,"$TORCH_DIR/lib" -ltorch_cpu -lc10
echo "built $REF_OUT (-march=$REF_MARCH)"

#!/usr/bin/env python3
"""Compiles every tests/dsl/*.txt and bench/dsl/*.txt program with galac and builds it (g++ over libtorch +
libgala_torch.so) into gala-gnn-acceleration-language_amd/progs/<name>/gala_prog, with the
IR next to it (ir.json) for the GPU parity tests.  Unchanged programs are not rebuilt.

    python tools/build_dsl_progs.py [-j 4] [program.txt ...]
"""
import argparse
import concurrent.futures as cf
import filecmp
import glob
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gala-gnn-acceleration-language_amd")
GALAC = os.path.join(PKG, "gala", "galac")
PROGS = os.path.join(PKG, "progs")


def build_one(src: str) -> str:
    name = os.path.splitext(os.path.basename(src))[0]
    out = os.path.join(PROGS, name)
    os.makedirs(out, exist_ok=True)
    with tempfile.TemporaryDirectory() as tmp:
        r = subprocess.run([GALAC, src, tmp, "--quiet", "--ir-json", os.path.join(tmp, "ir.json")],
                           capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(f"galac {src}: {r.stderr}")
        changed = False
        for f in ("gala.cpp", "Makefile", "ir.json"):
            dst = os.path.join(out, f)
            if not os.path.exists(dst) or not filecmp.cmp(os.path.join(tmp, f), dst, shallow=False):
                shutil.copy(os.path.join(tmp, f), dst)
                changed = True
    exe = os.path.join(out, "gala_prog")
    libs = [os.path.join(PKG, "gala", "libgala_torch.so"), os.path.join(PKG, "host", "gala_runtime.h"),
            os.path.join(PKG, "host", "gala_torch.h")]
    stale = changed or not os.path.exists(exe) or any(
        os.path.getmtime(l) > os.path.getmtime(exe) for l in libs)
    if stale:
        r = subprocess.run(["make", "-B", "-C", out], capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(f"build {name}: {r.stderr[-3000:]}")
    return f"{name}: {'built' if stale else 'up to date'}"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=4)
    ap.add_argument("programs", nargs="*")
    a = ap.parse_args(argv)
    srcs = a.programs or sorted(glob.glob(os.path.join(ROOT, "tests", "dsl", "*.txt")) +
                                glob.glob(os.path.join(ROOT, "bench", "dsl", "*.txt")))
    with cf.ThreadPoolExecutor(max_workers=a.j) as ex:
        for msg in ex.map(build_one, srcs):
            print(msg)
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""The reference's DSL corpus (tests/GALA-DSL, 114 programs) through the single-device path:
galac -> gala.cpp -> g++ over libgala_torch.so -> gala_prog, one program per structural
class (the same op graph and schedule flags; the classes of tests/test_dist_run_corpus_cpu.py),
each run for one epoch on the host-CPU backend (--device cpu) on a synthetic graph of its
dataset's shape scaled to about 1200 vertices, and its --dump checked against the float64
executor of its IR (tests/_ir_ref.py; forward, loss and weight gradients, the tolerance of
tests/_dsl_check.py).  Needs /root/reference (this container only); the programs are built
under a scratch directory, never in the repo, and only the summary is kept:

    python tools/corpus_progs.py [-j 8] [--out profiles/r03_corpus_progs_cpu.jsonl]
"""
import argparse
import concurrent.futures as cf
import glob
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gala-gnn-acceleration-language_amd")
GALAC = os.path.join(PKG, "gala", "galac")
CORPUS_DIR = "/root/reference/tests/GALA-DSL"
TARGET_N = 1200
sys.path[:0] = [os.path.join(ROOT, "tests"), PKG]


def classes(work):
    """{structure key: [(weight size, corpus-relative name, ir dict)]}."""
    out = {}
    for i, p in enumerate(sorted(glob.glob(os.path.join(CORPUS_DIR, "**", "*.txt"), recursive=True))):
        irp = os.path.join(work, f"ir_{i}.json")
        subprocess.run([GALAC, p, "--quiet", "--ir-json", irp], check=True, capture_output=True)
        ir = json.load(open(irp))["post"]
        s = {k: v for k, v in ir["sched"].items() if k not in ("dataset", "iterations", "feat_size", "label_size",
                                                                  "col_tile")}
        ops = tuple((n["op"], 0 if n["op"] == "FULL" else n["param"], n["graph"], tuple(n["in"])) for n in ir["nodes"])
        key = (json.dumps(s, sort_keys=True), ops, ir.get("num_graphs"))
        size = sum(int(w.get("in", 1)) * int(w.get("out", 1)) for w in ir["weights"]) * ir["sched"]["feat_size"]
        out.setdefault(key, []).append((size, os.path.relpath(p, CORPUS_DIR), ir))
    return out


def build_and_run(work, name, n_members, ir):
    from gala import dist_run
    tag = name.replace("/", "_")[:-4]
    d = os.path.join(work, tag)
    os.makedirs(d, exist_ok=True)
    t0 = time.time()
    r = subprocess.run([GALAC, os.path.join(CORPUS_DIR, name), d, "--quiet", "--ir-json", os.path.join(d, "ir.json")],
                       capture_output=True, text=True)
    if r.returncode:
        return {"program": name, "status": "galac failed", "detail": r.stderr[-500:]}
    r = subprocess.run(["make", "-B", "-C", d], capture_output=True, text=True)
    if r.returncode:
        return {"program": name, "status": "build failed", "detail": r.stderr[-800:]}
    t_build = time.time() - t0
    scale = min(1.0, TARGET_N / dist_run.dataset_shape(ir["sched"]["dataset"])[0])
    dump = os.path.join(d, "run.dump")
    r = subprocess.run([os.path.join(d, "gala_prog"), "--synthetic", "--seed", "3", "--scale", repr(scale),
                        "--device", "cpu", "--iters", "1", "--dump", dump], capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, OMP_NUM_THREADS="2"))
    if r.returncode:
        return {"program": name, "status": "run failed", "detail": r.stderr[-800:]}
    return {"program": name, "dump": dump, "ir": os.path.join(d, "ir.json"), "members": n_members,
            "dataset": ir["sched"]["dataset"], "scale": scale, "build_s": round(t_build, 1)}


def check(res):
    import _ir_ref as ref
    from _dsl_check import check_against_ir_file
    d = ref.read_dump(res.pop("dump"))
    try:
        check_against_ir_file(res.pop("ir"), d)
        res["status"] = "ok"
        res["checked"] = "forward, loss, weight gradients vs the float64 IR executor"
    except AssertionError as e:
        res["status"] = "mismatch"
        res["detail"] = str(e)[-800:]
    res["rows"] = int(len(d["rowptr"]) - 1)
    res["edges"] = int(d["col"].shape[0])
    return res


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_corpus_progs_cpu.jsonl"))
    a = ap.parse_args(argv)
    if not os.path.isdir(CORPUS_DIR):
        print("corpus_progs: the reference corpus is not present", file=sys.stderr)
        return 2
    with tempfile.TemporaryDirectory(prefix="gala_corpus_") as work:
        cls = classes(work)
        reps = [(min(m, key=lambda x: x[0]), len(m)) for m in cls.values()]
        print(f"{sum(n for _, n in reps)} programs in {len(reps)} structural classes; building in {work}",
              file=sys.stderr)
        with cf.ThreadPoolExecutor(max_workers=a.j) as ex:
            runs = list(ex.map(lambda rm: build_and_run(work, rm[0][1], rm[1], rm[0][2]), reps))
        out = [check(r) if "dump" in r else r for r in runs]
    with open(a.out, "w") as f:
        for r in out:
            f.write(json.dumps(r) + "\n")
    bad = [r for r in out if r["status"] != "ok"]
    print(f"{len(out) - len(bad)} of {len(out)} classes ok -> {a.out}", file=sys.stderr)
    for r in bad:
        print(r, file=sys.stderr)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())

"""CPU: the reference's DSL corpus (tests/GALA-DSL, 114 programs: GCN / GAT / GIN / SAGE on
six datasets plus the sampling, scalability, memory and speed-up ablations) runs unchanged
through galac -- as the generated single-device program and under the multi-rank runtime
gala.dist_run -- and each program computes what its IR means.

Only in this container: the corpus is read from /root/reference (it never travels to the
GPU box, and no copy of it is kept here), so the tests skip without it.

* every program compiles, and gala.dist_run accepts its post-pass IR on the row partition
  and, except the kernel-sampled ones, on the vertex cut;
* the programs fall into structural classes (the same op graph and schedule flags; they
  differ in dataset, widths and iteration counts).  One program of every class -- the one
  with the fewest weights -- runs one epoch on the host-CPU backend at world 1 on a
  synthetic graph of its dataset's shape scaled to about 1200 vertices, and its first
  forward, loss and weight gradients must equal the float64 executor of its IR
  (tests/_dist_check.py);
* the same representatives as generated programs (galac -> gala.cpp -> g++ over
  libgala_torch.so, built in a scratch directory by tools/corpus_progs.py) run one epoch on
  the host-CPU backend, their --dump checked the same way (tests/_dsl_check.py).
"""
import glob
import json
import os
import subprocess

import numpy as np
import pytest

from _dist_check import check_dist_dump

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "gala-gnn-acceleration-language_amd")
GALAC = os.path.join(PKG, "gala", "galac")
CORPUS = sorted(glob.glob("/root/reference/tests/GALA-DSL/**/*.txt", recursive=True))
TARGET_N = 1200

pytestmark = pytest.mark.skipif(not CORPUS, reason="reference DSL corpus not present")


def _compile(path, out):
    r = subprocess.run([GALAC, path, "--quiet", "--ir-json", str(out)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, (path, r.stderr)
    return json.loads(out.read_text())["post"]


def _classes(tmp_path):
    """{structure key: [(weights, name, ir path, ir)]} over the corpus."""
    out = {}
    for i, p in enumerate(CORPUS):
        irp = tmp_path / f"ir_{i}.json"
        ir = _compile(p, irp)
        s = {k: v for k, v in ir["sched"].items() if k not in ("dataset", "iterations", "feat_size", "label_size",
                                                                  "col_tile")}
        ops = tuple((n["op"], 0 if n["op"] == "FULL" else n["param"], n["graph"], tuple(n["in"])) for n in ir["nodes"])
        key = (json.dumps(s, sort_keys=True), ops, ir.get("num_graphs"))
        size = sum(int(w.get("in", 1)) * int(w.get("out", 1)) for w in ir["weights"]) * ir["sched"]["feat_size"]
        out.setdefault(key, []).append((size, os.path.relpath(p, "/root/reference/tests/GALA-DSL"), irp, ir))
    return out


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    return _classes(tmp_path_factory.mktemp("corpus"))


def test_corpus_is_accepted_by_the_multi_rank_runtime(corpus):
    from gala import dist_run
    progs = [m for v in corpus.values() for m in v]
    assert len(progs) == len(CORPUS) >= 100
    for _, name, _, ir in progs:
        dist_run.check_program(ir, "halo")
        if not ir["sched"]["kernel_sample"]:
            dist_run.check_program(ir, "vcut")
        assert dist_run.dataset_shape(ir["sched"]["dataset"]) is not None, name


def test_every_corpus_class_matches_its_ir_semantics(corpus, tmp_path, monkeypatch):
    """One program per structural class, world 1, host-CPU backend, against the float64 IR
    executor (forward, loss, weight gradients)."""
    from gala import dist_run
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("OMP_NUM_THREADS", "4")
    checked = []
    for key, members in corpus.items():
        _, name, irp, ir = min(members, key=lambda m: m[0])
        n0 = dist_run.dataset_shape(ir["sched"]["dataset"])[0]
        scale = min(1.0, TARGET_N / n0)
        dump = tmp_path / (name.replace("/", "_") + ".npz")
        lay = "vcut" if (len(checked) % 2 and not ir["sched"]["kernel_sample"]) else "halo"
        dist_run.main([str(irp), "--synthetic", "--scale", repr(scale), "--device", "cpu", "--iters", "1",
                       "--dump", str(dump), "--layout", lay])
        d = dict(np.load(dump))
        try:
            check_dist_dump(irp, d)
        except AssertionError as e:
            raise AssertionError(f"{name} ({lay}): {e}") from None
        checked.append(name)
    assert len(checked) == len(corpus) >= 25


def test_every_corpus_class_runs_as_a_generated_program(tmp_path):
    """tools/corpus_progs.py: one generated program per structural class, built and run on
    the host backend, forward / loss / weight gradients against the IR executor."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    import corpus_progs
    out = tmp_path / "corpus.jsonl"
    assert corpus_progs.main(["-j", "8", "--out", str(out)]) == 0
    rows = [json.loads(line) for line in out.read_text().splitlines()]
    assert len(rows) >= 25 and all(r["status"] == "ok" for r in rows)
    assert sum(r["members"] for r in rows) == len(CORPUS)


"""CPU: the galac-generated test programs run end to end on the host backend
(`--device cpu`: the operator mirror over libgala_cpu.so, torch CPU for the dense
layers) and match the float64 executor of their IR (tests/_dsl_check.py states the
tolerances).  Config 1 of BASELINE.json (Cora GCN on CPU libtorch) is
test_cora_gcn_inference_config1."""
import os
import subprocess

import numpy as np

import pytest

from _dsl_check import PKG, PROGS, RESULT, check_against_ir, check_against_ir_file, run_prog

BENCH_PROG = os.path.join(PKG, "progs", "gcn_cora_cpu", "gala_prog")


@pytest.mark.skipif(not PROGS, reason="generated programs not built (build() / tools/build_dsl_progs.py)")
@pytest.mark.parametrize("name", PROGS)
def test_program_on_cpu_matches_ir_semantics(name, tmp_path):
    _, d = run_prog(name, tmp_path, "--iters", "6", "--device", "cpu")
    check_against_ir(name, d)


@pytest.mark.skipif(not os.path.exists(BENCH_PROG), reason="bench/dsl programs not built")
def test_cora_gcn_inference_config1(tmp_path):
    """Config 1 (bench/dsl/gcn_cora_cpu.txt: Cora GCN-2, hidden 16, col_tile(100000), the
    gala_inference schedule) on the host backend: the run prints its timing / accuracy line,
    and its first epoch -- prediction, loss and weight gradients -- matches the float64
    executor of its own post-pass IR (tests/_dsl_check.py's tolerances), like every
    tests/dsl program."""
    from _ir_ref import read_dump
    dump = tmp_path / "cora.dump"
    r = subprocess.run([BENCH_PROG, "--synthetic", "--seed", "3", "--device", "cpu", "--iters", "10",
                        "--dump", str(dump)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    fwd, acc = map(float, r.stdout.strip().splitlines()[-1].split(","))
    assert fwd > 0 and 0.0 <= acc <= 100.0
    d = read_dump(str(dump))
    assert d["t_iden"].shape == (2708, 1433) and d["prediction"].shape == (2708, 7)
    check_against_ir_file(os.path.join(os.path.dirname(BENCH_PROG), "ir.json"), d)


def test_gpu_device_without_gpu_fails_loudly(tmp_path):
    """No silent fallback: the default device is the GPU, and without one the program stops."""
    if not PROGS:
        pytest.skip("generated programs not built")
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    exe = os.path.join(PKG, "progs", PROGS[0], "gala_prog")
    r = subprocess.run([exe, "--synthetic", "--iters", "1"], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "no GPU visible" in r.stderr


def test_npy_dataset_ids_out_of_range_fail_loudly(tmp_path):
    """from_files range-checks Adj_src / Adj_dst ids before narrowing them to int32: an id
    >= n (here 2^32 - 3, which wraps to -3, and n + 5, which would stay in int32 range but
    name no vertex) is refused with a message, never turned into another graph."""
    n = 50
    rng = np.random.default_rng(0)
    rows = np.sort(rng.integers(0, n, 200))
    cols = rng.integers(0, n, 200)
    exe = os.path.join(PKG, "progs", "gcn", "gala_prog")
    for bad in (2 ** 32 - 3, n + 5):
        data = tmp_path / f"Data{bad}"
        data.mkdir()
        c = cols.copy().astype(np.int64)
        c[7] = bad
        np.save(data / "Adj_src.npy", np.concatenate([[n, n], rows]).astype(np.uint32))
        np.save(data / "Adj_dst.npy", c.astype(np.uint32))
        np.save(data / "Feat.npy", np.zeros((n, 64), np.float32))
        np.save(data / "Lab.npy", np.zeros((n, 1), np.int64))
        for m in ("TnMsk", "VlMsk", "TsMsk"):
            np.save(data / f"{m}.npy", np.ones((n, 1), np.int32))
        r = subprocess.run([exe, "--data", str(data), "--iters", "1", "--device", "cpu"],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode != 0 and "vertex ids outside" in (r.stderr + r.stdout), r.stderr[-2000:]


def _directed_npy(path, n=500, m=3000, feat=64, classes=7, seed=11):
    """A directed graph (random arcs + self loops, so A^T != A) with features, labels and
    masks in the reference's npy format (tests/common.h:331-389)."""
    rng = np.random.default_rng(seed)
    src = np.concatenate([rng.integers(0, n, m), np.arange(n)]).astype(np.uint32)
    dst = np.concatenate([(src[:m] + rng.integers(1, 50, m)) % n, np.arange(n)]).astype(np.uint32)
    path.mkdir()
    np.save(path / "Adj_src.npy", np.concatenate([[n, n], src]).astype(np.uint32))
    np.save(path / "Adj_dst.npy", dst)
    np.save(path / "Feat.npy", rng.uniform(-1, 1, (n, feat)).astype(np.float32))
    np.save(path / "Lab.npy", rng.integers(0, classes, (n, 1)).astype(np.int64))
    train = rng.random(n) < 0.4
    np.save(path / "TnMsk.npy", train.astype(np.int32).reshape(-1, 1))
    np.save(path / "VlMsk.npy", np.zeros((n, 1), np.int32))
    np.save(path / "TsMsk.npy", (~train).astype(np.int32).reshape(-1, 1))


@pytest.mark.parametrize("name", ["gcn_directed", "gat_directed"])
def test_directed_program_on_a_directed_graph(name, tmp_path):
    """set_undirected(false) on a graph whose transpose differs: the backward runs on slot
    2g+1 = buildTranspose (GAT: the reference's chain on that pattern with the forward's
    alpha by edge position, common.h:835-894), on the host backend, against the IR executor
    (forward, loss, weight gradients)."""
    from _dsl_check import check_against_ir
    exe = os.path.join(PKG, "progs", name, "gala_prog")
    if not os.path.exists(exe):
        pytest.skip("generated programs not built")
    import json
    ir = json.load(open(os.path.join(PKG, "progs", name, "ir.json")))["post"]
    _directed_npy(tmp_path / "Data", feat=ir["sched"]["feat_size"], classes=ir["sched"]["label_size"])
    dump = tmp_path / "d.dump"
    r = subprocess.run([exe, "--data", str(tmp_path / "Data"), "--device", "cpu", "--seed", "3", "--iters", "1",
                        "--dump", str(dump)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    import _ir_ref as ref
    d = ref.read_dump(str(dump))
    rp = d["rowptr"]
    assert not np.array_equal(np.diff(rp), np.bincount(d["col"], minlength=len(rp) - 1))
    check_against_ir(name, d)


def test_program_on_a_matrix_market_graph(tmp_path):
    """--data FILE.mtx: a generated program on a Matrix Market graph (the reference's readSM
    semantics: 1-based entries, a symmetric file mirrored; the pattern is the adjacency) with
    synthetic node data; the graph is the one layout.load_mtx builds, and one epoch matches
    the IR executor."""
    from _dsl_check import check_against_ir
    from gala import layout
    import _ir_ref as ref
    rng = np.random.default_rng(8)
    n = 600
    r, c = rng.integers(1, n + 1, 2500), rng.integers(1, n + 1, 2500)
    pairs = np.unique(np.stack([np.maximum(r, c), np.minimum(r, c)], 1), axis=0)
    ent = [f"{a} {b}" for a, b in pairs if a != b] + [f"{i} {i}" for i in range(1, n + 1)]
    p = tmp_path / "g.mtx"
    p.write_text("\n".join(["%%MatrixMarket matrix coordinate pattern symmetric", "% test", f"{n} {n} {len(ent)}"]
                           + ent) + "\n")
    exe = os.path.join(PKG, "progs", "gcn", "gala_prog")
    dump = tmp_path / "d.dump"
    res = subprocess.run([exe, "--data", str(p), "--device", "cpu", "--seed", "3", "--iters", "1", "--dump",
                          str(dump)], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    d = ref.read_dump(str(dump))
    g = layout.load_mtx(str(p))
    np.testing.assert_array_equal(d["rowptr"], g.rowptr)
    np.testing.assert_array_equal(d["col"], g.col)
    check_against_ir("gcn", d)

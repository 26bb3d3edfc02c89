"""GPU: gala.dist_run (the multi-rank runtime of galac programs, BASELINE config 5) on the
MI355X through libgala_hip.so.

* one rank: the first forward of tests/dsl/gcn3.txt equals the float64 IR executor on the
  runner's graph, features and weights;
* two ranks sharing the one GPU over gloo (the box has one GPU; RCCL needs one device per
  rank): gathered predictions equal the one-rank predictions, the loss curve agrees.
"""
import pytest

from test_dist_run_cpu import _ir, _run, ref  # noqa: F401  (shared launch helpers)

import json
import os

import numpy as np
import torch

pytestmark = pytest.mark.gpu


def _run_gpu(ir, tmp_path, world, tag, iters=6, extra=(), backend="gloo"):
    import subprocess
    import sys
    from test_dist_run_cpu import PKG, ROOT, _free_port
    dump = tmp_path / f"{tag}.npz"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = PKG + os.pathsep + env.get("PYTHONPATH", "")
    env["GALA_DIST_BACKEND"] = backend
    cmd = [sys.executable]
    if world > 1:
        cmd += ["-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}", "--master-addr",
                "127.0.0.1", f"--master-port={_free_port()}", "-m", "gala.dist_run"]
    else:
        cmd += ["-m", "gala.dist_run"]
    cmd += [str(ir), "--synthetic", "--device", "cuda", "--iters", str(iters), "--dump", str(dump), *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    return dict(np.load(dump))


def test_dist_run_gpu_one_rank_matches_ir(tmp_path):
    from gala import dist_run
    ir_path = _ir("gcn3.txt", tmp_path)
    d = _run_gpu(ir_path, tmp_path, 1, "g1", iters=1)
    ir = ref.load_ir(str(ir_path))["post"]
    graphs = ref.Graphs(ir, d["rowptr"], d["col"], np.ones(len(d["rowptr"]) - 1, np.int32))
    X = torch.as_tensor(dist_run._hash_uniform(np.arange(len(d["rowptr"]) - 1), ir["sched"]["feat_size"], 3),
                        dtype=torch.float64)
    params = {k: torch.tensor(np.asarray(v), dtype=torch.float64) for k, v in json.loads(str(d["weights"])).items()}
    want = ref.run(ir, graphs, X, params)
    np.testing.assert_allclose(d["prediction"], want.detach().numpy(), rtol=1e-4, atol=1e-4)


def test_dist_run_gpu_two_ranks_match_one(tmp_path):
    ir_path = _ir("gcn3.txt", tmp_path)
    d1 = _run_gpu(ir_path, tmp_path, 1, "g1")
    d2 = _run_gpu(ir_path, tmp_path, 2, "g2")
    np.testing.assert_allclose(d2["prediction"], d1["prediction"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(d2["losses"], d1["losses"], rtol=1e-4, atol=1e-6)


def test_dist_run_gpu_vertex_cut_matches_one_rank(tmp_path):
    """`--layout vcut` on the HIP kernels: one rank (the class's own copy path) and two ranks
    sharing the GPU over gloo, against the one-rank halo run within fp32 rounding."""
    ir_path = _ir("gcn3.txt", tmp_path)
    d1 = _run_gpu(ir_path, tmp_path, 1, "g1")
    for world in (1, 2):
        dv = _run_gpu(ir_path, tmp_path, world, f"v{world}", extra=("--layout", "vcut"))
        np.testing.assert_allclose(dv["prediction"], d1["prediction"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(dv["losses"], d1["losses"], rtol=1e-4, atol=1e-6)


def test_dist_run_gpu_gat_program(tmp_path):
    """A GAT program (gat_heads: 4 heads) through the HIP kernels: the vertex cut at one rank
    against the float64 IR executor; two ranks sharing the GPU over gloo (the vertex cut with
    the dense and the sparse exchange, and the halo layout's HaloGat) against one rank."""
    from gala import dist_run
    ir_path = _ir("gat_heads.txt", tmp_path)
    d1 = _run_gpu(ir_path, tmp_path, 1, "g1", extra=("--layout", "vcut"))
    ir = ref.load_ir(str(ir_path))["post"]
    graphs = ref.Graphs(ir, d1["rowptr"], d1["col"], np.ones(len(d1["rowptr"]) - 1, np.int32))
    X = torch.as_tensor(dist_run._hash_uniform(np.arange(len(d1["rowptr"]) - 1), ir["sched"]["feat_size"], 3),
                        dtype=torch.float64)
    params = {k: torch.tensor(np.asarray(v), dtype=torch.float64) for k, v in json.loads(str(d1["weights"])).items()}
    want = ref.run(ir, graphs, X, params)
    np.testing.assert_allclose(d1["prediction"], want.detach().numpy(), rtol=1e-4, atol=1e-4)
    for extra in (("--layout", "vcut", "--exchange", "dense"), ("--layout", "vcut", "--exchange", "sparse"),
                  ("--layout", "halo")):
        d2 = _run_gpu(ir_path, tmp_path, 2, "g2" + extra[-1], extra=extra)
        np.testing.assert_allclose(d2["prediction"], d1["prediction"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(d2["losses"], d1["losses"], rtol=1e-4, atol=1e-6)


def _khop_induced(rowptr, col, seeds, hops):
    """Rows within `hops` of the seeds and the induced CSR on them (local ids): rows at
    distance < hops keep every edge, which is all a `hops`-layer forward of the seeds reads."""
    cur = np.unique(np.asarray(seeds, np.int64))
    allr = cur
    for _ in range(hops):
        nb = np.concatenate([col[rowptr[r]:rowptr[r + 1]] for r in cur]).astype(np.int64)
        cur = np.setdiff1d(np.unique(nb), allr)
        allr = np.union1d(allr, cur)
    loc = {int(r): i for i, r in enumerate(allr)}
    rp, cl = [0], []
    for r in allr:
        cs = [loc[int(c)] for c in col[rowptr[r]:rowptr[r + 1]] if int(c) in loc]
        cl += cs
        rp.append(len(cl))
    return allr, np.asarray(rp, np.int64), np.asarray(cl, np.int64)


@pytest.mark.timeout(500)
@pytest.mark.parametrize("scale,iters", [(0.1, 3), (1.0, 2)])
def test_dist_run_config5_shape_at_size(scale, iters, tmp_path):
    """Config 5's program (bench/dsl/gcn3_papers10.txt, GCN-3 hidden 128, 172 classes) at
    its own shape -- 11.1 M rows, the 10 % papers100M subset of
    tests/GALA-DSL/ablations/scalability/graph_10.txt (scale 1.0) -- and at 1.1 M rows
    (--scale 0.1), through the multi-rank runtime on the one GPU: the vertex cut over RCCL
    at world 1 (--dist: its reduce-scatters, or with --exchange sparse its uneven all-to-alls
    -- 5.7 GB per exchange at 11.1 M rows, cut into 512 MiB rounds -- and receive-CSR sums,
    run) against the halo layout's exact mode (sampled rows' predictions within 1e-5, the
    first loss within 1e-6, the curve within fp32 rounding), and the halo run's first forward
    against the float64 IR executor on sampled rows (their 3-hop induced subgraph, true
    degrees)."""
    from gala import dist_run
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ir_path = tmp_path / "p10.json"
    import subprocess
    from test_dist_run_cpu import GALAC
    r = subprocess.run([GALAC, os.path.join(root, "bench", "dsl", "gcn3_papers10.txt"), "--quiet", "--ir-json",
                        str(ir_path)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    common = ("--scale", str(scale), "--dump-stride", "997")
    dh = _run_gpu(ir_path, tmp_path, 1, "halo", iters=iters, extra=common)
    n = len(dh["rowptr"]) - 1
    assert n >= 11_000_000 * scale
    for exch in ("dense", "sparse"):
        dv = _run_gpu(ir_path, tmp_path, 1, "vcut_" + exch, iters=iters,
                      extra=common + ("--layout", "vcut", "--dist", "--exchange", exch), backend="nccl")
        np.testing.assert_array_equal(dv["rows"], dh["rows"])
        np.testing.assert_allclose(dv["prediction"], dh["prediction"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(dv["losses"][0], dh["losses"][0], rtol=1e-6, atol=0)
        np.testing.assert_allclose(dv["losses"], dh["losses"], rtol=1e-4, atol=1e-6)
    ir = ref.load_ir(str(ir_path))["post"]
    seeds = dh["rows"][:: max(len(dh["rows"]) // 6, 1)][:6]
    rowptr, col = dh["rowptr"].astype(np.int64), dh["col"]
    rows, rp, cl = _khop_induced(rowptr, col, seeds, 3)
    graphs = ref.Graphs(ir, rp, cl, np.ones(len(rows), np.int32))
    graphs.deg0 = torch.as_tensor(np.diff(rowptr)[rows].astype(np.float64)).view(-1, 1)   # true degrees
    X = torch.as_tensor(dist_run._hash_uniform(rows, ir["sched"]["feat_size"], 3), dtype=torch.float64)
    params = {k: torch.tensor(np.asarray(v), dtype=torch.float64) for k, v in json.loads(str(dh["weights"])).items()}
    want = ref.run(ir, graphs, X, params).detach().numpy()
    at = {int(r): i for i, r in enumerate(rows)}
    got_at = {int(r): i for i, r in enumerate(dh["rows"])}
    for s in seeds:
        np.testing.assert_allclose(dh["prediction"][got_at[int(s)]], want[at[int(s)]], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("prog,lay", [("gcn_ksample_dyn.txt", "halo"), ("gcn_ksample.txt", "halo"),
                                      ("gcn_gsample.txt", "vcut"), ("gcn_sparse.txt", "halo"),
                                      ("gcn3.txt", "vcut"), ("gat_heads.txt", "halo")])
def test_dist_run_gpu_programs_match_ir_with_gradients(prog, lay, tmp_path):
    """The HIP kernels under the multi-rank runtime at one rank: sampled (kernel, dynamic,
    graph), sparse-rewrite, GCN-3 on the vertex cut and the 4-head GAT on the row partition,
    against the float64 IR executor -- forward, loss and the first epoch's weight gradients."""
    from _dist_check import check_dist_dump
    ir_path = _ir(prog, tmp_path)
    d = _run_gpu(ir_path, tmp_path, 1, "g1", iters=1, extra=("--layout", lay))
    check_dist_dump(ir_path, d)


@pytest.mark.parametrize("lay", ["halo", "vcut"])
def test_dist_run_gpu_directed_program(lay, tmp_path):
    """A directed program on a directed npy graph: the backward over A^T's partition."""
    from _dist_check import check_dist_dump
    from test_dist_run_cpu import _directed_dataset
    ir_path = _ir("gcn_directed.txt", tmp_path)
    inputs = _directed_dataset(tmp_path / "Data", ir_path)
    d = _run_gpu(ir_path, tmp_path, 1, "g1", iters=1, extra=("--layout", lay, "--data", str(tmp_path / "Data")))
    check_dist_dump(ir_path, d, inputs)


def test_dist_run_gpu_dynamic_sampling_two_ranks_bit_identical(tmp_path):
    """Dynamic kernel sampling over two ranks sharing the GPU: the same (ra, rb) draws and
    the first forward bit-identical to one rank."""
    ir_path = _ir("gcn_ksample_dyn.txt", tmp_path)
    d1 = _run_gpu(ir_path, tmp_path, 1, "g1")
    d2 = _run_gpu(ir_path, tmp_path, 2, "g2")
    np.testing.assert_array_equal(d2["samples"], d1["samples"])
    np.testing.assert_array_equal(d2["prediction"], d1["prediction"])
    np.testing.assert_allclose(d2["losses"], d1["losses"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("prog,lay", [("gcn_directed.txt", "halo"), ("gcn_directed.txt", "vcut"),
                                      ("gcn_ksample_dyn.txt", "halo"), ("gcn_sparse.txt", "vcut")])
def test_dist_run_gpu_rccl_world_one_matches_no_collectives(prog, lay, tmp_path):
    """RCCL at world 1 (--dist: every collective of the layout runs, the transposed
    partitions' included): a one-rank collective moves rows unchanged, so the run is
    bit-identical to the same run without collectives."""
    extra = ("--layout", lay)
    if prog == "gcn_directed.txt":
        from test_dist_run_cpu import _directed_dataset
        _directed_dataset(tmp_path / "Data", _ir(prog, tmp_path))
        extra += ("--data", str(tmp_path / "Data"))
    ir_path = _ir(prog, tmp_path)
    d0 = _run_gpu(ir_path, tmp_path, 1, "plain", iters=3, extra=extra)
    d1 = _run_gpu(ir_path, tmp_path, 1, "rccl", iters=3, extra=extra + ("--dist",), backend="nccl")
    np.testing.assert_array_equal(d1["prediction"], d0["prediction"])
    np.testing.assert_array_equal(d1["samples"], d0["samples"])
    np.testing.assert_allclose(d1["losses"], d0["losses"], rtol=1e-6, atol=0)

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


def _run_gpu(ir, tmp_path, world, tag, iters=6, extra=()):
    import subprocess
    import sys
    from test_dist_run_cpu import PKG, ROOT, _free_port
    dump = tmp_path / f"{tag}.npz"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = PKG + os.pathsep + env.get("PYTHONPATH", "")
    env["GALA_DIST_BACKEND"] = "gloo"
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
    """A GAT program (gat_heads: 4 heads) on the vertex cut through the HIP kernels: one rank
    against the float64 IR executor, two ranks sharing the GPU over gloo (dense and sparse
    exchange) against one rank."""
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
    for ex in ("dense", "sparse"):
        d2 = _run_gpu(ir_path, tmp_path, 2, f"g2{ex}", extra=("--layout", "vcut", "--exchange", ex))
        np.testing.assert_allclose(d2["prediction"], d1["prediction"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(d2["losses"], d1["losses"], rtol=1e-4, atol=1e-6)

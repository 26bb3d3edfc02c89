"""CPU: the galac-generated test programs run end to end on the host backend
(`--device cpu`: the operator mirror over libgala_cpu.so, torch CPU for the dense
layers) and match the float64 executor of their IR (tests/_dsl_check.py states the
tolerances).  Config 1 of BASELINE.json (Cora GCN on CPU libtorch) is
test_cora_gcn_inference_config1."""
import os
import subprocess

import numpy as np

import pytest

from _dsl_check import PKG, PROGS, RESULT, check_against_ir, run_prog

BENCH_PROG = os.path.join(PKG, "progs", "gcn_cora_cpu", "gala_prog")


@pytest.mark.skipif(not PROGS, reason="generated programs not built (build() / tools/build_dsl_progs.py)")
@pytest.mark.parametrize("name", PROGS)
def test_program_on_cpu_matches_ir_semantics(name, tmp_path):
    _, d = run_prog(name, tmp_path, "--iters", "6", "--device", "cpu")
    check_against_ir(name, d)


@pytest.mark.skipif(not os.path.exists(BENCH_PROG), reason="bench/dsl programs not built")
def test_cora_gcn_inference_config1():
    r = subprocess.run([BENCH_PROG, "--synthetic", "--device", "cpu", "--iters", "10"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    fwd, acc = map(float, r.stdout.strip().splitlines()[-1].split(","))
    assert fwd > 0 and 0.0 <= acc <= 100.0


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

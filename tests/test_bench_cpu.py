"""CPU: bench.py's launch contract (the driver runs `python bench.py --gpus N`).

* `--gpus 2` without a launcher starts its own two ranks (torch.distributed.run on
  127.0.0.1) and prints ONE JSON line with n_gpus 2, strong scaling of the one graph and
  a `comm` block naming the chosen partitioning mode.  `--device cpu` runs the same code
  on the host-CPU backend over gloo: a plumbing check, not a measurement.
* Under a launcher, WORLD_SIZE must equal --gpus.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    return env


def _run_ranks(args, env, timeout=600):
    """bench.py with self-launched gloo ranks, run once: a rank that aborts in teardown
    ("terminate called without an active exception") fails the test."""
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout, env=env,
                          cwd=ROOT)


def _json_lines(out: str):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def test_bench_self_launches_ranks():
    r = _run_ranks(["--gpus", "2", "--device", "cpu", "--scale", "0.002", "--steps", "2", "--warmup", "1",
                    "--calib-steps", "1"], _env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout                 # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["value"] > 0
    gat = d["gat"]                                    # the GAT layer: halo and vertex-cut layouts timed
    assert gat["value"] > 0 and set(gat["candidates_ms_per_step"]) >= {"halo", "halo-overlap", "vcut"}
    assert gat["layout"].split()[0] in gat["candidates_ms_per_step"]
    assert d["unit"] == "edges/s" and d["steps"] == 2 and d["warmup"] == 1
    c = d["comm"]
    assert c["mode"] in c["candidates_ms_per_step"]
    assert set(c["candidates_ms_per_step"]) >= {"halo-exact", "halo-overlap", "vcut", "vcut-pipe"}
    assert c["halo_bytes_per_aggregation_per_rank"] > 0 and c["exchange_ms_per_aggregation"] > 0
    assert c["exchange_GBps_per_rank"] > 0
    assert d["config"]["edges"] > 0 and "weak" in d and d["weak"]["value"] > 0
    assert d["roofline"]["alg_bytes_per_launch"] > 0
    # the skewed family strong-scaled too, with its own candidates and chosen layout
    rm = d["rmat"]
    assert rm["value"] > 0 and rm["comm"]["mode"] in rm["comm"]["candidates_ms_per_step"]
    assert "R-MAT" in rm["graph"] and 0.0 <= rm["comm"]["vcut_touched_fraction"] <= 1.0
    assert "rehearsal" in c["rccl_note"]          # gloo: labelled as a rehearsal, not RCCL
    # the family that shards naturally: a row partition with a point-to-point halo of the
    # band's boundary rows only
    bd = d["banded"]
    assert bd["value"] > 0 and bd["comm"]["halo_layout"] == "p2p" and "banded" in bd["graph"]
    assert bd["comm"]["halo_bytes_per_aggregation_per_rank"] < c["halo_bytes_per_aggregation_per_rank"]
    # the largest message each collective kind sent (max over ranks) and its rounds
    m = c["messages"]
    assert m["cut_at_bytes"] == 1 << 29
    assert {"all_gather", "reduce_scatter"} <= set(m)
    for kind, st in m.items():
        if kind == "cut_at_bytes":
            continue
        assert st["calls"] > 0 and st["max_rounds"] >= 1 and st["max_payload_bytes"] >= st["max_call_bytes"] > 0
        if kind in ("all_to_all", "p2p"):
            assert st["max_call_bytes"] <= m["cut_at_bytes"]


def test_bench_eight_ranks():
    """The driver's N = 8 launch shape (8 self-launched ranks, here gloo on the host): one line
    with n_gpus 8, every family and field present, every partition of the 8-way split built."""
    env = _env()
    env["OMP_NUM_THREADS"] = "1"
    r = _run_ranks(["--gpus", "8", "--device", "cpu", "--scale", "0.002", "--steps", "2", "--warmup", "1",
                    "--calib-steps", "1"], env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == 8 and d["value"] > 0 and d["config"]["parallelism"].endswith("x8 (gloo)")
    assert all(k in d and d[k]["value"] > 0 for k in ("gat", "rmat", "banded", "weak"))
    assert not d["budget"]["skipped_for_time"] and set(d["budget"]["phase_s"]) == {"uniform", "gat", "rmat",
                                                                                     "banded", "weak"}


def test_bench_budget_keeps_the_headline():
    """--budget-s far below what the run needs: the N = 2 line still carries the headline
    (its first candidate timed, the others and every secondary field skipped, agreed over
    the ranks), with the skips listed under budget.skipped_for_time."""
    r = _run_ranks(["--gpus", "2", "--device", "cpu", "--scale", "0.002", "--steps", "2", "--warmup", "1",
                    "--calib-steps", "1", "--budget-s", "0.01"], _env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["ms_per_step"] > 0
    assert list(d["comm"]["candidates_ms_per_step"]) == ["halo-exact"]
    b = d["budget"]
    assert b["budget_s"] == 0.01 and b["skipped_for_time"]
    skipped = " ".join(b["skipped_for_time"])
    for field in ("gat field", "rmat family", "banded family", "weak field", "uniform candidate vcut"):
        assert field in skipped
    assert not any(k in d for k in ("gat", "rmat", "banded", "weak"))
    assert b["phase_s"]["uniform"] > 0


def test_bench_single_rank_line():
    r = subprocess.run([sys.executable, BENCH, "--device", "cpu", "--scale", "0.002", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline", "--banded"],
                       capture_output=True, text=True, timeout=600, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    (d,) = _json_lines(r.stdout)
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert "rmat" in d and d["rmat"]["value"] > 0 and d["rmat"]["roofline"]["alg_bytes_per_launch"] > 0
    assert d["banded"]["value"] > 0 and "banded" in d["banded"]["graph"]


def test_bench_rejects_world_mismatch():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--device", "cpu", "--scale", "0.002"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_bench_partitioned_path_on_one_rank():
    """GALA_BENCH_DIST=1: the strong-scaling path on one rank without a launcher (the GPU
    suite runs it over RCCL; here gloo on the host-CPU backend)."""
    env = _env()
    env["GALA_BENCH_DIST"] = "1"
    r = subprocess.run([sys.executable, BENCH, "--device", "cpu", "--scale", "0.002", "--steps", "2",
                        "--warmup", "1", "--calib-steps", "1"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    (d,) = _json_lines(r.stdout)
    assert d["n_gpus"] == 1 and d["comm"]["backend"] == "gloo" and d["value"] > 0


def _write_npy_dataset(d, n=1500, m=6000, seed=4):
    """A small dataset in the reference's on-disk format (scripts/Data/gala_export_npy.py:
    100-112): Adj_src.npy = uint32 [n_rows, n_cols, src...], Adj_dst.npy = uint32 [dst...],
    symmetric edges + self loops."""
    import numpy as np
    rng = np.random.default_rng(seed)
    u, v = rng.integers(0, n, m), rng.integers(0, n, m)
    src = np.concatenate([u, v, np.arange(n)]).astype(np.uint32)
    dst = np.concatenate([v, u, np.arange(n)]).astype(np.uint32)
    np.save(os.path.join(d, "Adj_src.npy"), np.concatenate([[n, n], src]).astype(np.uint32))
    np.save(os.path.join(d, "Adj_dst.npy"), dst)
    return n, src.shape[0]


def test_bench_real_data(tmp_path):
    """--data DIR: the headline step runs on the dataset's graph (read through the runtime's
    npy loader) and the line names it; one rank and two self-launched ranks."""
    n, e = _write_npy_dataset(str(tmp_path))
    for extra in ((), ("--gpus", "2", "--calib-steps", "1", "--no-weak", "--no-gat")):
        r = _run_ranks(["--device", "cpu", "--data", str(tmp_path), "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-rmat", *extra], _env())
        assert r.returncode == 0, r.stderr[-3000:]
        (d,) = _json_lines(r.stdout)
        assert d["config"]["n_vertices"] == n and d["config"]["edges"] == e
        assert d["data"].startswith("real: ") and str(tmp_path) in d["data"]


def test_bench_matrix_market_graph(tmp_path):
    """--data FILE.mtx: the headline step on a Matrix Market graph (symmetric pattern file,
    mirrored as the reference's readSM does), one rank."""
    import numpy as np
    rng = np.random.default_rng(5)
    n, m = 1200, 5000
    r = rng.integers(1, n + 1, m)
    c = rng.integers(1, n + 1, m)
    lo, hi = np.maximum(r, c), np.minimum(r, c)
    keep = np.unique(np.stack([lo, hi], 1), axis=0)
    lines = ["%%MatrixMarket matrix coordinate pattern symmetric", f"{n} {n} {keep.shape[0] + n}"]
    lines += [f"{a} {b}" for a, b in keep if a != b] + [f"{i} {i}" for i in range(1, n + 1)]
    lines[1] = f"{n} {n} {len(lines) - 2}"
    p = tmp_path / "g.mtx"
    p.write_text("\n".join(lines) + "\n")
    from gala import layout
    g = layout.load_mtx(str(p))
    res = subprocess.run([sys.executable, BENCH, "--device", "cpu", "--data", str(p), "--steps", "2", "--warmup", "1",
                          "--no-cpu-baseline", "--no-rmat"], capture_output=True, text=True, timeout=600, env=_env(),
                         cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    (d,) = _json_lines(res.stdout)
    assert d["config"]["n_vertices"] == n and d["config"]["edges"] == g.nnz
    assert "Matrix Market" in d["data"]



def test_traffic_is_withheld_when_the_kernel_sources_changed(tmp_path, monkeypatch):
    """bench.py reports a kernel's PMC bytes (profiles/traffic.json) only while the sources its
    pass ran on are unchanged: a digest mismatch or a missing digest withholds the number and
    lists the kernel under traffic_withheld_stale."""
    sys.path.insert(0, ROOT)
    import bench
    committed = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
    key = next(k for k in committed["kernels"] if k.startswith("void gala::k_spmm_rowgroup<4, 8, 1, 4"))
    entry = committed["kernels"][key]
    assert entry.get("sources_sha256"), "the committed PMC summary records its source digests"
    # the committed summary against this tree: fresh
    monkeypatch.setattr(bench, "TRAFFIC_STALE", [])
    assert bench.load_traffic("k_spmm_rowgroup<4, 8, 1, 4, false, false, false, false>") == \
        float(entry["hbm_bytes_per_launch"])
    assert bench.TRAFFIC_STALE == []
    # one source digest off, and none at all: withheld
    fake_root = tmp_path / "root"
    (fake_root / "profiles").mkdir(parents=True)
    os.symlink(os.path.join(ROOT, "gala-gnn-acceleration-language_amd"), fake_root / "gala-gnn-acceleration-language_amd")
    for digests in ({**entry["sources_sha256"], "gala-gnn-acceleration-language_amd/csrc/spmm.hip": "0" * 64}, None):
        e = dict(entry)
        if digests is None:
            e.pop("sources_sha256")
        else:
            e["sources_sha256"] = digests
        json.dump({"kernels": {key: e}}, open(fake_root / "profiles" / "traffic.json", "w"))
        monkeypatch.setattr(bench, "ROOT", str(fake_root))
        monkeypatch.setattr(bench, "TRAFFIC_STALE", [])
        assert bench.load_traffic("k_spmm_rowgroup<4, 8, 1, 4, false, false, false, false>") is None
        assert bench.TRAFFIC_STALE == ["k_spmm_rowgroup<4, 8, 1, 4, false, false, false, false>"]

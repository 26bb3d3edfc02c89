#!/usr/bin/env python3
"""Generates tests/golden/*.npz from the REFERENCE's own CPU code.

Run in the build container (needs /root/reference and oracle/_ref/libgala_ref.so, built
by oracle/build_ref.sh from the reference headers in place):

    python tests/golden/make_golden.py

Every expected output below is produced by the reference implementation itself:
  CSR layout     readSM_npy32's CSRCMatrix::build + set_all(1)
                 (tests/common.h:331-366, src/formats/csrc_matrix.h:148-376,413-421)
  column tiles   static_ord_col_breakpoints + ord_col_tiling_torch
                 (src/ops/tiling.h:1594-1608, 222-283)
  sampling       inplace_sample_graph_ab(n, 5, 7) (src/ops/tiling.h:454-508)
  SpMM           gSpMM + wsumAgg (src/ops/aggregators.h:12-31,55-127)
  subgraphs      getMaskSubgraphs + buildTranspose (src/utils/common.h:26-129)
Inputs are seeded numpy draws, stored in the fixture next to the outputs.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as orc  # noqa: E402


def coo_uniform(n, m_undirected, seed):
    """Symmetric random edges + one self loop per vertex (gala_export_npy.py:73-74 shape)."""
    rng = np.random.default_rng(seed)
    u = rng.integers(0, n, m_undirected)
    v = rng.integers(0, n, m_undirected)
    src = np.concatenate([u, v, np.arange(n)]).astype(np.int32)
    dst = np.concatenate([v, u, np.arange(n)]).astype(np.int32)
    perm = rng.permutation(src.shape[0])          # unsorted input order
    return src[perm], dst[perm]


def coo_powerlaw(n, m, seed):
    """Skewed (Zipf-like) symmetric graph + self loops."""
    rng = np.random.default_rng(seed)
    w = 1.0 / np.arange(1, n + 1) ** 0.9
    w /= w.sum()
    u = rng.choice(n, m, p=w)
    v = rng.integers(0, n, m)
    src = np.concatenate([u, v, np.arange(n)]).astype(np.int32)
    dst = np.concatenate([v, u, np.arange(n)]).astype(np.int32)
    perm = rng.permutation(src.shape[0])
    return src[perm], dst[perm]


def coo_directed_sparse(n, m, seed):
    """Directed, no self loops, rows >= n/2 empty (edge case for build/tile/SpMM)."""
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n // 2, m).astype(np.int32)
    dst = rng.integers(0, n, m).astype(np.int32)
    return src, dst


def make(name, n, src, dst, F_list, weighted_F, integer_x, tiles, samples):
    rp, col, val = orc.ref_csr_build(n, n, src, dst)
    out = {"n": np.int64(n), "src": src, "dst": dst, "rowptr": rp, "col": col,
           "csr_val": val}
    g = orc.Graph(n, n, rp, col, None)
    rng = np.random.default_rng(1234)
    Fmax = max(F_list)
    if integer_x:
        X = rng.integers(-8, 9, (n, Fmax)).astype(np.float32)
    else:
        X = rng.uniform(-1, 1, (n, Fmax)).astype(np.float32)
    out["X"] = X
    w = np.random.default_rng(99).uniform(0, 1, col.shape[0]).astype(np.float32)
    out["w"] = w
    for F in F_list:
        out[f"Y_F{F}"] = orc.ref_gspmm(g, np.ascontiguousarray(X[:, :F]))
    for F in weighted_F:
        gw = orc.Graph(n, n, rp, col, w)
        out[f"Yw_F{F}"] = orc.ref_gspmm(gw, np.ascontiguousarray(X[:, :F]))
    for cpp in tiles:
        t = orc.ref_col_tile(g, cpp)
        out[f"tile{cpp}_rowptr"] = t.rowptr
        out[f"tile{cpp}_col"] = t.col
        out[f"tile{cpp}_bounds"] = t.bounds
    for ns in samples:
        s = orc.ref_sample_ab(g, ns, 5, 7)
        out[f"sample{ns}_rowptr"] = s.rowptr
        out[f"sample{ns}_col"] = s.col
    # training-subgraph levels for a 30% train mask (codegen/common.h:480-492)
    mask = (np.random.default_rng(5).uniform(0, 1, n) < 0.3).astype(np.float32)
    out["train_mask"] = mask
    for lvl, (frp, fcol, trp, tcol) in enumerate(orc.ref_mask_subgraphs(g, mask, 3)):
        out[f"sub{lvl}_rowptr"], out[f"sub{lvl}_col"] = frp, fcol
        out[f"subT{lvl}_rowptr"], out[f"subT{lvl}_col"] = trp, tcol
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{path}: N={n} E={col.shape[0]} keys={len(out)} {os.path.getsize(path)/1024:.0f} KiB")


def main():
    assert orc.ref_available(), "build oracle/_ref first (oracle/build_ref.sh)"
    s, d = coo_uniform(2708, 5278, seed=42)                       # Cora-shaped
    make("cora_uniform", 2708, s, d, [1, 7, 16, 47], [16, 47], False, [903, 1000], [20])
    s, d = coo_powerlaw(1024, 8000, seed=7)
    make("powerlaw", 1024, s, d, [32, 40, 64, 100, 128], [32, 100], True, [342, 100], [20, 5])
    s, d = coo_directed_sparse(600, 2500, seed=3)
    make("directed_sparse", 600, s, d, [8, 33], [8], False, [200, 64], [])


if __name__ == "__main__":
    main()

"""Shared test graphs (seeded, small enough for the oracle to finish in seconds)."""
from __future__ import annotations

import numpy as np

import oracle as orc
from gala import layout


def to_oracle(g: layout.HostGraph, val=None, heads=1) -> orc.Graph:
    v = g.val if val is None else val
    return orc.Graph(g.n_rows, g.n_cols, g.rowptr, g.col, v, g.n_seg, g.bounds, heads)


def cora_like(seed=42) -> layout.HostGraph:
    # N=2708, 5278 undirected edges + N self loops = 13264 stored edges
    return layout.gen_graph("uniform", 2708, 5278, seed)


def powerlaw(n=4096, m=30000, seed=7) -> layout.HostGraph:
    return layout.gen_graph("rmat", n, m, seed)


def banded(n=3000, width=40, per_row=6, seed=5) -> layout.HostGraph:
    """Symmetric graph with locality: every edge joins vertices at most `width` apart, plus
    self loops (a few vertex ranges touch each row: the sparse vertex-cut exchange)."""
    rng = np.random.default_rng(seed)
    u = np.repeat(np.arange(n, dtype=np.int64), per_row)
    v = np.clip(u + rng.integers(-width, width + 1, u.shape[0]), 0, n - 1)
    src = np.concatenate([u, v, np.arange(n)]).astype(np.int32)
    dst = np.concatenate([v, u, np.arange(n)]).astype(np.int32)
    return layout.csr_build(n, n, src, dst)


def with_empty_rows(n=700, m=3000, seed=3) -> layout.HostGraph:
    """Directed random graph (no self loops) with a block of empty rows + one heavy row."""
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n // 2, m).astype(np.int32)       # rows >= n/2 empty
    dst = rng.integers(0, n, m).astype(np.int32)
    heavy = np.full(900, 5, np.int32)                        # row 5: >= 900 edges
    src = np.concatenate([src, heavy])
    dst = np.concatenate([dst, rng.integers(0, n, 900).astype(np.int32)])
    return layout.csr_build(n, n, src, dst)


def long_row_graph(seed=3) -> layout.HostGraph:
    """Mean degree ~600 (hub threshold 8 * 600 > 4096): rows of 4 500 edges (above the row
    order's counting-sort cap, below the threshold) beside real hub rows of 9 000-12 000."""
    rng = np.random.default_rng(seed)
    n = 2000
    deg = rng.integers(450, 750, n)
    deg[[5, 700, 1500, 1999]] = 4500
    deg[[3, 900, 1200]] = [9000, 12000, 9000]
    src = np.repeat(np.arange(n), deg).astype(np.int32)
    dst = rng.integers(0, n, src.shape[0]).astype(np.int32)
    return layout.csr_build(n, n, src, dst)


def features(n, F, seed=1234, integer=False):
    rng = np.random.default_rng(seed)
    if integer:
        return rng.integers(-8, 9, (n, F)).astype(np.float32)
    return rng.uniform(-1, 1, (n, F)).astype(np.float32)


def edge_values(nnz, heads=1, seed=99, lo=0.0, hi=1.0):
    rng = np.random.default_rng(seed)
    return rng.uniform(lo, hi, nnz * heads).astype(np.float32)

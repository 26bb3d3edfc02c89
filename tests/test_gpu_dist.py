"""GPU: the partitioned aggregation's HIP path on one device (ranks simulated in-process;
the all-gather is a concatenation of the boundary blocks).  Checks the two-segment
local/halo SpMM launch sequence of gala/dist.py against the oracle on the assembled
global graph."""
import numpy as np
import pytest
import torch

import oracle as orc
from gala import dist as gdist
from gala import ops

pytestmark = pytest.mark.gpu


def _assert_matches_oracle(g, X, norm, got_rows, r0):
    """The vertex cut's owner rows against the ORACLE's GCN aggregation of the whole graph
    (norm * A (norm * X), orc_gspmm order) at north_star's tolerance: |err| <= 1e-4 abs +
    1e-4 rel -- an anchor that does not go through the one-GPU HIP result."""
    want = orc.spmm(orc.Graph(g.n_rows, g.n_cols, g.rowptr, g.col), X.cpu().numpy(),
                    src_scale=norm.cpu().numpy(), dst_scale=norm.cpu().numpy())[r0:r0 + got_rows.shape[0]]
    np.testing.assert_allclose(got_rows.cpu().numpy(), want, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("world", [2, 4])
def test_simulated_ranks_match_global_oracle(world):
    n, E, F = 3000, 40000, 32
    parts = [gdist.make_partition(r, world, n, E, cut_frac=0.15, boundary_frac=0.1, seed=3)
             for r in range(world)]
    b = parts[0].b
    rng = np.random.default_rng(0)
    Xg = rng.uniform(-1, 1, (world * n, F)).astype(np.float32)
    G = gdist.global_reference_graph(parts)
    norm_g = (1.0 / np.sqrt(G.degrees().astype(np.float32))).astype(np.float32)
    ref = orc.spmm(orc.Graph(G.n_rows, G.n_cols, G.rowptr, G.col), Xg, src_scale=norm_g, dst_scale=norm_g)

    Xs = []
    segs, norms = [], []
    for p in parts:
        full = ops.DeviceGraph.from_host(p.graph)
        norm = ops.degree(full, power=-0.5)
        norms.append(norm)
        segs.append([ops.DeviceGraph.from_host(gdist.segment_view(p.graph, s)) for s in range(2)])
        X = torch.from_numpy(Xg[p.rank * n:(p.rank + 1) * n]).cuda()
        buf = torch.empty((p.n_cols, F), device="cuda")
        ops.row_broadcast(norm, X, out=buf[:n])
        Xs.append(buf)
    halo = torch.cat([x[:b] for x in Xs])           # the all-gather
    outs = []
    for p, buf, sg, norm in zip(parts, Xs, segs, norms):
        buf[n:] = halo
        Y = torch.empty((n, F), device="cuda")
        ops.spmm(sg[0], buf, dst_scale=norm, out=Y)
        ops.spmm(sg[1], buf, dst_scale=norm, out=Y, accum=True)
        outs.append(Y)
    got = torch.cat(outs).cpu().numpy()
    np.testing.assert_allclose(got, ref, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("kind", ["uniform", "rmat"])
def test_partitioned_graph_matches_one_gpu(world, kind):
    """partition_graph's layout through the HIP SpMM, ranks simulated in-process (the halo
    exchange is a gather of the scaled features by global id).  exact mode (one SpMM over
    the monotone global -> Xs remap) is bit-identical to the one-GPU aggregation, hub
    rows included (the partition keeps the whole graph's split threshold); overlap mode
    (own edges, then halo edges accumulated) agrees to fp32 rounding."""
    from gala import layout
    g = layout.gen_graph(kind, 6000, 60000, seed=4)
    F = 32
    X = torch.from_numpy(np.random.default_rng(2).uniform(-1, 1, (g.n_rows, F)).astype(np.float32)).cuda()
    dg = ops.DeviceGraph.from_host(g)
    norm = ops.degree(dg, power=-0.5)
    Xs_g = ops.row_broadcast(norm, X)
    ref = ops.spmm(dg, Xs_g, dst_scale=norm)
    split_seen = dg.split_rows
    for p in range(world):
        pt = gdist.partition_graph(g, p, world, halo_mode="p2p")
        r0, r1 = pt.r0, pt.r0 + pt.n
        gg = ops.DeviceGraph.from_host(pt.graph, split=pt.split_threshold)
        split_seen -= gg.split_rows
        n_p = ops.degree(gg, power=-0.5)
        assert torch.equal(n_p, norm[r0:r1])
        Xs = Xs_g[torch.from_numpy(pt.xs_to_global()).cuda()]       # the simulated exchange
        ops.row_broadcast(n_p, X[r0:r1], out=Xs[pt.own_slice])
        Y = ops.spmm(gg, Xs, dst_scale=n_p)
        assert torch.equal(Y, ref[r0:r1])
        og = ops.DeviceGraph.from_host(pt.own_graph, split=pt.split_threshold)
        hg = ops.DeviceGraph.from_host(pt.halo_graph, split=pt.split_threshold)
        Y2 = ops.spmm(og, Xs, dst_scale=n_p)
        ops.spmm(hg, Xs, dst_scale=n_p, out=Y2, accum=True)
        torch.testing.assert_close(Y2, ref[r0:r1], rtol=1e-5, atol=1e-6)
    assert split_seen == 0      # the partitions split exactly the whole graph's hub rows


@pytest.mark.parametrize("world,chunks", [(2, 1), (3, 4)])
@pytest.mark.parametrize("kind", ["uniform", "rmat"])
def test_dense_halo_matches_one_gpu(world, chunks, kind):
    """The all-gather ("dense") halo layout, ranks simulated in-process: the padded table is
    filled from the global scaled features through xs_to_global (what the chunked
    all-gathers deliver).  One SpMM over the rank's rows is bit-identical to one GPU for any
    chunking; the overlapped own + per-chunk accumulation agrees to fp32 rounding."""
    from gala import layout
    g = layout.gen_graph(kind, 6000, 60000, seed=4)
    F = 32
    X = torch.from_numpy(np.random.default_rng(2).uniform(-1, 1, (g.n_rows, F)).astype(np.float32)).cuda()
    dg = ops.DeviceGraph.from_host(g)
    norm = ops.degree(dg, power=-0.5)
    Xs_g = ops.row_broadcast(norm, X)
    ref = ops.spmm(dg, Xs_g, dst_scale=norm)
    for p in range(world):
        pt = gdist.partition_graph(g, p, world, halo_mode="dense", chunks=chunks)
        r0, r1 = pt.r0, pt.r0 + pt.n
        gg = ops.DeviceGraph.from_host(pt.graph, split=pt.split_threshold)
        n_p = ops.degree(gg, power=-0.5)
        assert torch.equal(n_p, norm[r0:r1])
        x2g = torch.from_numpy(pt.xs_to_global()).cuda()
        table = torch.zeros((pt.n_cols, F), device="cuda")
        valid = x2g >= 0
        table[valid] = Xs_g[x2g[valid]]
        for j0, j1, x0 in pt.own_blocks():              # own rows written by the rank itself
            ops.row_broadcast(n_p[j0:j1], X[r0 + j0:r0 + j1], out=table[x0:x0 + j1 - j0])
        Y = ops.spmm(gg, table, dst_scale=n_p)
        assert torch.equal(Y, ref[r0:r1])
        Y2 = ops.spmm(ops.DeviceGraph.from_host(pt.groups[0], split=pt.split_threshold), table, dst_scale=n_p)
        for h in pt.groups[1:]:
            ops.spmm(ops.DeviceGraph.from_host(h, split=pt.split_threshold), table, dst_scale=n_p, out=Y2,
                     accum=True)
        torch.testing.assert_close(Y2, ref[r0:r1], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("world,chunks", [(2, 1), (3, 4), (4, 2)])
@pytest.mark.parametrize("kind", ["uniform", "rmat"])
def test_vertex_cut_matches_one_gpu(world, chunks, kind):
    """Column ownership (gala/vertex_cut.py), ranks simulated in-process: every rank's chunk
    SpMMs write partial rows over its own columns only; the reduce-scatter is the sum of the
    partial buffers over ranks, block `owner` to the owner.  norm * sum agrees with the
    one-GPU aggregation to fp32 rounding; degrees from the owned rows' offsets are exact."""
    from gala import layout, vertex_cut as vc
    g = layout.gen_graph(kind, 6000, 60000, seed=5)
    F = 32
    X = torch.from_numpy(np.random.default_rng(3).uniform(-1, 1, (g.n_rows, F)).astype(np.float32)).cuda()
    dg = ops.DeviceGraph.from_host(g)
    norm = ops.degree(dg, power=-0.5)
    ref = ops.spmm(dg, ops.row_broadcast(norm, X), dst_scale=norm)
    parts = [vc.vertex_cut_partition(g, p, world, chunks=chunks) for p in range(world)]
    c = parts[0].block
    total = torch.zeros((chunks * world * c, F), device="cuda")
    norms = []
    for pt in parts:
        r0, r1 = pt.r0, pt.r0 + pt.n
        n_p = ops.degree(ops.DeviceGraph.from_host(pt.deg_graph, split=False), power=-0.5)
        assert torch.equal(n_p, norm[r0:r1])
        norms.append(n_p)
        Xs = ops.row_broadcast(n_p, X[r0:r1])
        rows = world * c
        for k, h in enumerate(pt.chunk_graphs):
            total[k * rows:(k + 1) * rows] += ops.spmm(ops.DeviceGraph.from_host(h, split=pt.split_threshold), Xs)
    for q, pt in enumerate(parts):
        S = torch.cat([total[k * world * c + q * c:k * world * c + (q + 1) * c] for k in range(chunks)])[:pt.n]
        got = ops.row_broadcast(norms[q], S)
        torch.testing.assert_close(got, ref[pt.r0:pt.r0 + pt.n], rtol=1e-5, atol=1e-6)
        _assert_matches_oracle(g, X, norm, got, pt.r0)


def test_aggregator_classes_on_one_rank():
    """DistAggregator / VertexCutAggregator through HipBackend at world 1 (no collectives):
    the row partition is bit-identical, the chunked vertex cut within fp32 rounding."""
    from gala import layout, vertex_cut as vc
    from gala.backend import HipBackend
    g = layout.gen_graph("rmat", 5000, 50000, seed=6)
    F = 32
    be = HipBackend("cuda")
    X = torch.from_numpy(np.random.default_rng(4).uniform(-1, 1, (g.n_rows, F)).astype(np.float32)).cuda()
    dg = ops.DeviceGraph.from_host(g)
    norm = ops.degree(dg, power=-0.5)
    ref = ops.spmm(dg, ops.row_broadcast(norm, X), dst_scale=norm)
    agg = gdist.DistAggregator(gdist.partition_graph(g, 0, 1), F, be, None, exact=True)
    Y = torch.empty_like(X)
    agg(X, Y)
    assert torch.equal(Y, ref)
    agg2 = gdist.DistAggregator(gdist.partition_graph(g, 0, 1), F, be, None, exact=False)
    Y2 = torch.empty_like(X)
    agg2(X, Y2)
    assert torch.equal(Y2, ref)                       # one group: the own edges are all edges
    vagg = vc.VertexCutAggregator(vc.vertex_cut_partition(g, 0, 1, chunks=3), F, be, None)
    Y3 = torch.empty_like(X)
    vagg(X, Y3)
    torch.testing.assert_close(Y3, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("world,chunks", [(1, 2), (2, 1), (3, 4)])
@pytest.mark.parametrize("heads,F", [(1, 32), (8, 256)])
def test_vertex_cut_gat_matches_one_gpu(world, chunks, heads, F):
    """REF GAT forward with column ownership, ranks simulated in-process: every rank's
    GALA_GAT_PARTIAL launches over its own columns (aL of all rows = the all-gather);
    adding the ranks' partial rows and softmax sums (the reduce-scatters) and normalising
    equals the one-GPU fused forward and the oracle within the tolerance."""
    from gala import layout, vertex_cut as vc
    import oracle as orc_
    g = layout.gen_graph("uniform", 3000, 20000, seed=9)
    rng = np.random.default_rng(5)
    aL = rng.uniform(-1, 1, (g.n_rows, heads)).astype(np.float32)
    aR = rng.uniform(-1, 1, (g.n_rows, heads)).astype(np.float32)
    X = rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32)
    dg = ops.DeviceGraph.from_host(g)
    Y1 = ops.gat_fwd(dg, torch.from_numpy(aL).cuda(), torch.from_numpy(aR).cuda(), torch.from_numpy(X).cuda(),
                     heads=heads)
    parts = [vc.vertex_cut_partition(g, p, world, chunks=chunks) for p in range(world)]
    c, rows = parts[0].block, world * parts[0].block
    U = torch.zeros((chunks * rows, F), device="cuda")
    S = torch.zeros((chunks * rows, heads), device="cuda")
    # aL of every row in the partial graphs' (chunk, owner, row) layout
    aL_rows = torch.zeros((chunks * rows, heads), device="cuda")
    for pt in parts:
        for j0, j1 in [(k * c, min((k + 1) * c, pt.n)) for k in range(chunks)]:
            if j1 > j0:
                k = j0 // c
                aL_rows[k * rows + pt.rank * c:k * rows + pt.rank * c + (j1 - j0)] = \
                    torch.from_numpy(aL[pt.r0 + j0:pt.r0 + j1]).cuda()
    for pt in parts:
        own = slice(pt.r0, pt.r0 + pt.n)
        aRp, Xp = torch.from_numpy(aR[own].copy()).cuda(), torch.from_numpy(X[own].copy()).cuda()
        for k, h in enumerate(pt.chunk_graphs):
            gk = ops.DeviceGraph.from_host(h, split=pt.split_threshold)
            Uk, Sk = ops.gat_fwd_partial(gk, aL_rows[k * rows:(k + 1) * rows].contiguous(), Xp, aR=aRp, heads=heads)
            U[k * rows:(k + 1) * rows] += Uk
            S[k * rows:(k + 1) * rows] += Sk.view(-1, heads)
    D = F // heads
    for pt in parts:
        Uo = torch.cat([U[k * rows + pt.rank * c:k * rows + (pt.rank + 1) * c] for k in range(chunks)])[:pt.n]
        So = torch.cat([S[k * rows + pt.rank * c:k * rows + (pt.rank + 1) * c] for k in range(chunks)])[:pt.n]
        Y = (Uo.view(pt.n, heads, D) / (So + 1e-12).view(pt.n, heads, 1)).reshape(pt.n, F)
        torch.testing.assert_close(Y, Y1[pt.r0:pt.r0 + pt.n], rtol=1e-5, atol=1e-6)
    if world == 1:   # the class itself, on the HIP backend
        from gala.backend import HipBackend
        gat = vc.VertexCutGat(parts[0], F, heads, HipBackend("cuda"), None)
        Yc = gat(torch.from_numpy(aL).cuda(), torch.from_numpy(aR).cuda(), torch.from_numpy(X).cuda())
        torch.testing.assert_close(Yc, Y1, rtol=1e-5, atol=1e-6)
    Yr, _ = orc_.gat_fwd(orc_.Graph(g.n_rows, g.n_cols, g.rowptr, g.col), aL, aR, X, heads=heads)
    np.testing.assert_allclose(Y1.cpu().numpy(), Yr, atol=1e-4, rtol=1e-4)


def test_bench_partitioned_path_over_rccl_one_rank():
    """bench.py's strong-scaling path (every candidate layout, the weak-scaling field) on one
    rank with the RCCL backend (GALA_BENCH_DIST=1): the collectives' tensor contracts
    (device tensors, in-place all-gather blocks, reduce-scatter blocks, the max-reduce of
    the step time) go through RCCL itself.  The box has one GPU, so this is world 1."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "GALA_DIST_BACKEND")}
    env["GALA_BENCH_DIST"] = "1"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--scale", "0.05", "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=200, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-4000:]
    (d,) = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert d["n_gpus"] == 1 and d["scaling"] == "strong" and d["comm"]["backend"] == "nccl"
    assert set(d["comm"]["candidates_ms_per_step"]) >= {"halo-exact", "halo-overlap", "vcut", "vcut-pipe"}
    assert d["value"] > 0 and d["weak"]["value"] > 0 and d["gat"]["value"] > 0
    assert set(d["gat"]["candidates_ms_per_step"]) == {"halo", "halo-overlap", "vcut"}   # every GAT layout on RCCL


@pytest.mark.parametrize("world,chunks", [(1, 2), (2, 1), (3, 4)])
@pytest.mark.parametrize("heads,F", [(1, 32), (8, 256)])
def test_vertex_cut_gat_training_matches_one_gpu(world, chunks, heads, F):
    """The vertex-cut GAT training pair, ranks simulated in-process on the HIP kernels:
    gala_gat_fwd_partial_stats_f32 over every rank's columns, the partials added (the
    reduce-scatter) and normalised by the owner give the one-GPU gala_gat_fwd_stats_f32's
    Y, Ym, q and sma; the backward's partial P = sum p dY[col] (the partial forward on dY)
    times q gives the one-GPU row-statistics backward's dX, and d_aL from the owner's rows
    alone (an edgeless graph) its d_aL -- all within fp32 rounding.  world 1 also runs the
    VertexCutGat class itself."""
    from gala import layout, vertex_cut as vc
    g = layout.gen_graph("uniform", 3000, 20000, seed=9)
    rng = np.random.default_rng(6)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    aL = rng.uniform(-1, 1, (g.n_rows, heads)).astype(np.float32)
    aR = rng.uniform(-1, 1, (g.n_rows, heads)).astype(np.float32)
    X = rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32)
    dY = rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32)
    dg = ops.DeviceGraph.from_host(g)
    Y1, q1, Ym1, sma1 = ops.gat_fwd_stats(dg, cu(aL), cu(X), aR=cu(aR), heads=heads)
    dX1, daL1 = ops.gat_bwd_stats(dg, cu(aL), cu(aR), cu(dY), q1, Y1, Ym1, sma1, heads=heads)
    parts = [vc.vertex_cut_partition(g, p, world, chunks=chunks) for p in range(world)]
    c, rows = parts[0].block, world * parts[0].block
    aL_rows = torch.zeros((chunks * rows, heads), device="cuda")
    for pt in parts:
        for k in range(chunks):
            j0, j1 = k * c, min((k + 1) * c, pt.n)
            if j1 > j0:
                aL_rows[k * rows + pt.rank * c:k * rows + pt.rank * c + (j1 - j0)] = cu(aL[pt.r0 + j0:pt.r0 + j1])
    acc = {n_: torch.zeros((chunks * rows, F if n_ in ("U", "Um", "P") else heads), device="cuda")
           for n_ in ("U", "Um", "S", "M", "P")}
    for pt in parts:
        own = slice(pt.r0, pt.r0 + pt.n)
        for k, h in enumerate(pt.chunk_graphs):
            gk = ops.DeviceGraph.from_host(h, split=pt.split_threshold)
            al_k = aL_rows[k * rows:(k + 1) * rows].contiguous()
            U, S, Um, M = ops.gat_fwd_partial_stats(gk, al_k, cu(X[own]), aR=cu(aR[own]), heads=heads)
            P, _ = ops.gat_fwd_partial(gk, al_k, cu(dY[own]), aR=cu(aR[own]), heads=heads)
            for n_, t in (("U", U), ("Um", Um), ("S", S), ("M", M), ("P", P)):
                acc[n_][k * rows:(k + 1) * rows] += t.view(rows, -1)
    D = F // heads
    for pt in parts:
        sl = slice(pt.r0, pt.r0 + pt.n)
        o = {n_: torch.cat([t[k * rows + pt.rank * c:k * rows + (pt.rank + 1) * c] for k in range(chunks)])[:pt.n]
             for n_, t in acc.items()}
        q = 1.0 / (o["S"] + 1e-12)
        sc = lambda T: (T.view(pt.n, heads, D) * q.view(pt.n, heads, 1)).reshape(pt.n, F)  # noqa: E731
        Y, Ym, sma = sc(o["U"]), sc(o["Um"]), o["M"] * q
        torch.testing.assert_close(Y, Y1[sl], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(Ym, Ym1[sl], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(q.reshape(-1), q1.view(-1, heads)[sl].reshape(-1), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(sma.reshape(-1), sma1.view(-1, heads)[sl].reshape(-1), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(sc(o["P"]), dX1[sl], rtol=1e-5, atol=1e-6)
        eg = ops.DeviceGraph.from_host(layout.HostGraph(pt.n, pt.n, np.zeros(pt.n + 1, np.int32),
                                                        np.zeros(0, np.int32)), split=False)
        _, daL = ops.gat_bwd_stats(eg, cu(aL[sl]), cu(aR[sl]), cu(dY[sl]), q.contiguous(), Y, Ym,
                                   sma.contiguous(), heads=heads)
        torch.testing.assert_close(daL, daL1.view(-1, heads)[sl].reshape(-1), rtol=1e-4, atol=1e-4)
    # the own vertices' recomputed logits (gala_gat_fwd_partial_stats_ex_f32 with self_col):
    # every rank's chunks write exactly the one-GPU statistics forward's aR_out of its rows
    wR0 = cu(rng.uniform(-0.5, 0.5, F).astype(np.float32))
    bR0 = cu(rng.uniform(-0.5, 0.5, heads).astype(np.float32))
    *_, aR0 = ops.gat_fwd_stats(dg, cu(aL), cu(X), wR=wR0, bR=bR0, heads=heads, want_aR=True)
    for pt in parts:
        own = slice(pt.r0, pt.r0 + pt.n)
        got = torch.full((pt.n, heads), float("nan"), device="cuda")
        for k, h in enumerate(pt.chunk_graphs):
            gk = ops.DeviceGraph.from_host(h, split=pt.split_threshold)
            ops.gat_fwd_partial_stats(gk, aL_rows[k * rows:(k + 1) * rows].contiguous(), cu(X[own]), wR=wR0,
                                      bR=bR0, heads=heads, self_col=cu(pt.self_cols(k)), aR_out=got)
        assert torch.equal(got.reshape(-1), aR0.view(-1, heads)[own].reshape(-1))
    if world == 1:
        from gala.backend import HipBackend
        gat = vc.VertexCutGat(parts[0], F, heads, HipBackend("cuda"), None)
        Yc = gat.forward_train(cu(aL), cu(aR), cu(X))
        dXc, daLc = gat.backward(cu(dY))
        torch.testing.assert_close(Yc, Y1, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(dXc, dX1, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(daLc.reshape(-1), daL1, rtol=1e-4, atol=1e-4)
        # the source logits recomputed from X inside the partial kernel (the DSL's shape)
        wR = cu(rng.uniform(-0.5, 0.5, F).astype(np.float32))
        bR = cu(rng.uniform(-0.5, 0.5, heads).astype(np.float32))
        Y2, q2, Ym2, sma2, aR2 = ops.gat_fwd_stats(dg, cu(aL), cu(X), wR=wR, bR=bR, heads=heads, want_aR=True)
        dX2, daL2 = ops.gat_bwd_stats(dg, cu(aL), aR2, cu(dY), q2, Y2, Ym2, sma2, heads=heads)
        Yr = gat.forward_train(cu(aL), None, cu(X), wR, bR)
        assert torch.equal(gat.saved[1].reshape(-1), aR2)   # the forward's own-vertex logits, bit for bit
        dXr, daLr, _, _ = gat.backward(cu(dY))       # dX includes the path through aR = X wR + bR
        dX2 = ops.head_attn_bwd(daL2.view(-1, heads), wR, heads=heads, dX=dX2.clone())
        torch.testing.assert_close(Yr, Y2, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(dXr, dX2, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(daLr.reshape(-1), daL2, rtol=1e-4, atol=1e-4)


def test_bench_self_launch_two_ranks_on_one_gpu_gloo():
    """`bench.py --gpus 2` as the driver runs it (no launcher: it starts its own two ranks)
    on the HIP kernels, the two ranks sharing the box's one GPU over gloo: exactly one JSON
    line on stdout, strong scaling of the one graph, every layout candidate timed, and the
    GAT layer over the vertex cut."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["GALA_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--scale", "0.02", "--steps",
                        "2", "--warmup", "1", "--no-weak"], capture_output=True, text=True, timeout=220, env=env,
                       cwd=root)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["comm"]["backend"] == "gloo"
    assert set(d["comm"]["candidates_ms_per_step"]) >= {"halo-exact", "halo-overlap", "vcut", "vcut-pipe"}
    assert d["value"] > 0 and d["gat"]["value"] > 0
    assert set(d["gat"]["candidates_ms_per_step"]) >= {"halo", "halo-overlap", "vcut"}
    rm = d["rmat"]                                     # the skewed family at n_gpus 2
    assert rm["value"] > 0 and rm["comm"]["mode"] in rm["comm"]["candidates_ms_per_step"]
    bd = d["banded"]                                   # and the one that shards naturally
    assert bd["value"] > 0 and bd["comm"]["mode"] in bd["comm"]["candidates_ms_per_step"]


@pytest.mark.parametrize("world,chunks", [(2, 1), (3, 2), (4, 3)])
@pytest.mark.parametrize("kind", ["banded", "rmat"])
def test_vertex_cut_sparse_exchange_matches_one_gpu(world, chunks, kind):
    """The sparse (DCSR) vertex-cut exchange, ranks simulated in-process on the HIP kernels:
    every rank's SpMMs write only the destination rows it holds edges of, the all-to-all is
    the re-slicing of those blocks by (chunk, source rank), and the owner's receive-CSR SpMM
    (norm fused) equals the one-GPU aggregation to fp32 rounding."""
    from gala import layout, vertex_cut as vc
    from _graphs import banded
    g = banded(n=6000, width=60) if kind == "banded" else layout.gen_graph("rmat", 6000, 60000, seed=5)
    F = 32
    X = torch.from_numpy(np.random.default_rng(3).uniform(-1, 1, (g.n_rows, F)).astype(np.float32)).cuda()
    dg = ops.DeviceGraph.from_host(g)
    norm = ops.degree(dg, power=-0.5)
    ref = ops.spmm(dg, ops.row_broadcast(norm, X), dst_scale=norm)
    parts = [vc.vertex_cut_partition(g, p, world, chunks=chunks, exchange="sparse") for p in range(world)]
    sends = []
    for pt in parts:
        Xs = ops.row_broadcast(norm[pt.r0:pt.r0 + pt.n], X[pt.r0:pt.r0 + pt.n])
        blocks = []
        for k, h in enumerate(pt.sparse.send_graphs):
            Yk = ops.spmm(ops.DeviceGraph.from_host(h, split=pt.split_threshold), Xs)
            off = np.concatenate([[0], np.cumsum(pt.sparse.send_counts[k])])
            blocks.append([Yk[off[q]:off[q + 1]] for q in range(world)])
        sends.append(blocks)
    for pt in parts:
        recv = torch.cat([sends[q][k][pt.rank] for k in range(chunks) for q in range(world)])
        if recv.shape[0] == 0:
            recv = torch.zeros((1, F), device="cuda")
        got = ops.spmm(ops.DeviceGraph.from_host(pt.sparse.recv_graph, split=False), recv,
                       dst_scale=norm[pt.r0:pt.r0 + pt.n])
        torch.testing.assert_close(got, ref[pt.r0:pt.r0 + pt.n], rtol=1e-5, atol=1e-6)
        _assert_matches_oracle(g, X, norm, got, pt.r0)


@pytest.mark.parametrize("heads,F", [(1, 32), (8, 256)])
def test_vertex_cut_sparse_classes_on_one_rank(heads, F):
    """VertexCutAggregator and the VertexCutGat training pair with the sparse exchange at
    world 1 on the HIP backend (the receive-CSR SpMMs, the aL index gather, the attention
    Linear's backward) against the one-GPU operators."""
    from gala import layout, vertex_cut as vc
    from gala.backend import HipBackend
    g = layout.gen_graph("rmat", 4000, 40000, seed=8)
    be = HipBackend("cuda")
    rng = np.random.default_rng(7)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    X = cu(rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32))
    dY = cu(rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32))
    aL = cu(rng.uniform(-1, 1, (g.n_rows, heads)).astype(np.float32))
    wR = cu(rng.uniform(-0.5, 0.5, F).astype(np.float32))
    bR = cu(rng.uniform(-0.5, 0.5, heads).astype(np.float32))
    dg = ops.DeviceGraph.from_host(g)
    norm = ops.degree(dg, power=-0.5)
    ref = ops.spmm(dg, ops.row_broadcast(norm, X), dst_scale=norm)
    pt = vc.vertex_cut_partition(g, 0, 1, chunks=2, exchange="sparse")
    agg = vc.VertexCutAggregator(pt, F, be, None)
    Y = torch.empty_like(X)
    agg(X, Y)
    torch.testing.assert_close(Y, ref, rtol=1e-5, atol=1e-6)
    Y2, q2, Ym2, sma2, aR2 = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=heads, want_aR=True)
    dX2, daL2 = ops.gat_bwd_stats(dg, aL, aR2, dY, q2, Y2, Ym2, sma2, heads=heads)
    dX2 = ops.head_attn_bwd(daL2.view(-1, heads), wR, heads=heads, dX=dX2.clone())
    gat = vc.VertexCutGat(pt, F, heads, be, None)
    Yr = gat.forward_train(aL, None, X, wR, bR)
    assert torch.equal(gat.saved[1].reshape(-1), aR2)       # own-vertex logits from the compact rows
    dXr, daLr, dW, db = gat.backward(dY)
    torch.testing.assert_close(Yr, Y2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(daLr.reshape(-1), daL2, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dXr, dX2, rtol=1e-4, atol=1e-5)
    D = F // heads
    g64 = daL2.view(-1, heads).double()
    torch.testing.assert_close(dW.double(), (g64.repeat_interleave(D, 1) * X.double()).sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db.double(), g64.sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("world,halo", [(1, "p2p"), (2, "dense"), (3, "p2p"), (4, "dense")])
@pytest.mark.parametrize("kind,heads,F", [("uniform", 8, 256), ("rmat", 1, 32), ("rmat", 4, 64)])
def test_halo_gat_bit_identical_to_one_gpu(world, halo, kind, heads, F):
    """The halo GAT pair, ranks simulated in-process on the HIP kernels: rank p's table holds
    every row its edges read (the exchange is a gather by global id), and
    gala_gat_{fwd,bwd}_stats_ex_f32 over its rows (self_col = the own block of the table,
    dY_rows = the table's own rows) give Y, q, Ym, sma, aR_out, dX and d_aL BIT-identical
    to the one-GPU pair -- hub-row chunks included (the whole graph's threshold).  world 1
    also runs the HaloGat class."""
    from gala import layout
    g = layout.gen_graph(kind, 5000, 50000, seed=12)
    rng = np.random.default_rng(9)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    aL = rng.uniform(-1, 1, (g.n_rows, heads)).astype(np.float32)
    X = rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32)
    dY = rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32)
    wR = cu(rng.uniform(-0.5, 0.5, F).astype(np.float32))
    bR = cu(rng.uniform(-0.5, 0.5, heads).astype(np.float32))
    dg = ops.DeviceGraph.from_host(g)                    # the whole graph's hub plan
    Y1, q1, Ym1, sma1, aR1 = ops.gat_fwd_stats(dg, cu(aL), cu(X), wR=wR, bR=bR, heads=heads, want_aR=True)
    dX1, daL1 = ops.gat_bwd_stats(dg, cu(aL), aR1, cu(dY), q1, Y1, Ym1, sma1, heads=heads)
    dXl1, _ = ops.gat_bwd_stats(dg, cu(aL), aR1, cu(dY), q1, Y1, Ym1, sma1, heads=heads, wR=wR)
    for p in range(world):
        pt = gdist.partition_graph(g, p, world, halo_mode=halo)
        own = slice(pt.r0, pt.r0 + pt.n)
        x2g = torch.from_numpy(np.maximum(pt.xs_to_global(), 0)).cuda()
        Xs, dYs = cu(X)[x2g].contiguous(), cu(dY)[x2g].contiguous()
        x0 = pt.own_offset()
        gp = ops.DeviceGraph.from_host(pt.graph, split=pt.split_threshold)
        sc = torch.arange(x0, x0 + pt.n, dtype=torch.int32, device="cuda")
        As = torch.full((pt.n_cols, heads), float("nan"), device="cuda")
        Y, q, Ym, sma = ops.gat_fwd_stats(gp, cu(aL[own]), Xs, wR=wR, bR=bR, heads=heads, self_col=sc, aR_out=As)
        assert torch.equal(Y, Y1[own]) and torch.equal(Ym, Ym1[own])
        assert torch.equal(q.view(-1, heads), q1.view(-1, heads)[own])
        assert torch.equal(sma.view(-1, heads), sma1.view(-1, heads)[own])
        assert torch.equal(As[x0:x0 + pt.n], aR1.view(-1, heads)[own])
        Aall = aR1.view(-1, heads)[x2g].contiguous()         # the exchanged logits table
        dX, daL = ops.gat_bwd_stats(gp, cu(aL[own]), Aall, dYs, q, Y, Ym, sma, heads=heads,
                                    dY_rows=dYs[x0:x0 + pt.n])
        assert torch.equal(dX, dX1[own]) and torch.equal(daL.view(-1, heads), daL1.view(-1, heads)[own])
        # the attention Linear folded into the dX store over the gathered table + dY_rows
        # (gala_gat_bwd_stats_linear_f32 as HaloGat.backward runs it)
        dXl, daLl = ops.gat_bwd_stats(gp, cu(aL[own]), Aall, dYs, q, Y, Ym, sma, heads=heads,
                                      dY_rows=dYs[x0:x0 + pt.n], wR=wR)
        assert torch.equal(dXl, dXl1[own]) and torch.equal(daLl, daL)
        if world == 1:
            from gala.backend import HipBackend
            be = HipBackend("cuda")
            hg = gdist.HaloGat(pt, F, heads, be, None)
            Yc = hg.forward_train(cu(aL), None, cu(X), wR, bR)
            dXc, daLc = hg.backward(cu(dY), linear=False)
            assert torch.equal(Yc, Y1) and torch.equal(dXc, dX1) and torch.equal(daLc.reshape(-1), daL1)
            Yc = hg.forward_train(cu(aL), None, cu(X), wR, bR)
            dXc, daLc, dW, db = hg.backward(cu(dY), linear=True)
            dW1, db1 = be.head_linear_grads(cu(X), daL1.view(-1, heads), heads)
            assert torch.equal(dXc, dXl1) and torch.equal(daLc.reshape(-1), daL1)
            assert torch.equal(dW, dW1) and torch.equal(db, db1)


@pytest.mark.parametrize("world,halo,chunks", [(1, "p2p", 1), (2, "dense", 1), (3, "p2p", 1), (4, "dense", 1),
                                               (2, "dense", 3), (4, "dense", 4)])
@pytest.mark.parametrize("kind,heads,F", [("uniform", 8, 256), ("rmat", 1, 32), ("rmat", 4, 64)])
def test_halo_gat_overlap_matches_one_gpu(world, halo, chunks, kind, heads, F):
    """HaloGatOverlap, ranks simulated in-process (comm None; the tables pre-filled with the
    rows the exchange would deliver): own-column partial statistics, then every halo chunk
    continued from them (gala_gat_fwd_continue_f32; 1-4 chunks of a dense table) -- Y, dX,
    d_aL within fp32 rounding of the one-GPU pair (each row's sums grouped per range), the
    own logits written bit for bit."""
    from gala import layout
    from gala.backend import HipBackend
    g = layout.gen_graph(kind, 5000, 50000, seed=12)
    rng = np.random.default_rng(9)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    aL = cu(rng.uniform(-1, 1, (g.n_rows, heads)).astype(np.float32))
    X = cu(rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32))
    dY = cu(rng.uniform(-1, 1, (g.n_rows, F)).astype(np.float32))
    wR = cu(rng.uniform(-0.5, 0.5, F).astype(np.float32))
    bR = cu(rng.uniform(-0.5, 0.5, heads).astype(np.float32))
    dg = ops.DeviceGraph.from_host(g)
    Y1, q1, Ym1, sma1, aR1 = ops.gat_fwd_stats(dg, aL, X, wR=wR, bR=bR, heads=heads, want_aR=True)
    dX1, daL1 = ops.gat_bwd_stats(dg, aL, aR1, dY, q1, Y1, Ym1, sma1, heads=heads)
    A1 = aR1.view(-1, heads)
    for p in range(world):
        pt = gdist.partition_graph(g, p, world, halo_mode=halo, chunks=chunks)
        own = slice(pt.r0, pt.r0 + pt.n)
        x2g = torch.from_numpy(np.maximum(pt.xs_to_global(), 0)).cuda()
        hg = gdist.HaloGatOverlap(pt, F, heads, HipBackend("cuda"), None)
        hg.Xs.copy_(X[x2g])
        hg.dYs.copy_(dY[x2g])
        hg.As.copy_(A1[x2g])
        sc = hg.self_col.long()
        hg.As[sc] = float("nan")                           # the forward writes the own rows' logits
        Y = hg.forward_train(aL[own], None, X[own], wR, bR)
        assert torch.equal(hg.As[sc], A1[own])
        dX, daL = hg.backward(dY[own], linear=False)
        torch.testing.assert_close(Y, Y1[own], rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(dX, dX1[own], rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(daL.reshape(-1), daL1.view(-1, heads)[own].reshape(-1), rtol=1e-4, atol=1e-4)

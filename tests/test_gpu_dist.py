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
        pt = gdist.partition_graph(g, p, world)
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

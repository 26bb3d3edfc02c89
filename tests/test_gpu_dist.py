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

"""TEST INFRASTRUCTURE: checks a gala.dist_run --dump (one rank) against the float64
executor of the program's IR (tests/_ir_ref.py): the first forward's predictions and loss
on the training rows, and the first epoch's weight gradients, with the tolerance of
tests/_dsl_check.py (fp32 vs float64)."""
import json

import numpy as np
import torch

import _ir_ref as ref


def synthetic_inputs(ir, n, seed=3):
    """dist_run's synthetic features, labels and training rows (its counter hashes)."""
    from gala import dist_run
    s = ir["sched"]
    rows = np.arange(n)
    frac = dist_run.dataset_shape(s["dataset"])[4]
    train = (dist_run._hash_int(rows, seed + 2, 1 << 20) < int(frac * (1 << 20))) | (rows == 0)
    return (dist_run._hash_uniform(rows, s["feat_size"], seed), dist_run._hash_int(rows, seed + 1, s["label_size"]),
            train)


def check_dist_dump(ir_path, d, inputs=None):
    """A one-rank dump against the float64 IR executor on the same graph, features and
    weights: the first forward's predictions and loss, and the first epoch's weight
    gradients (the tolerance of tests/_dsl_check.py).  Kernel sampling uses the (ra, rb)
    the runner drew for its first forward."""
    ir = ref.load_ir(str(ir_path))["post"]
    n = len(d["rowptr"]) - 1
    X, labels, train = inputs if inputs is not None else synthetic_inputs(ir, n)
    ra, rb = (int(v) for v in d["samples"][0]) if d["samples"].shape[0] else (5, 7)
    graphs = ref.Graphs(ir, d["rowptr"], d["col"], train.astype(np.int32), ra=ra, rb=rb)
    W = json.loads(str(d["weights"]))
    name = lambda k: k[:-2] if k.endswith(".0") else k   # noqa: E731  (eps ParameterList -> eps<k>)
    params = {name(k): torch.tensor(np.asarray(v), dtype=torch.float64, requires_grad=True) for k, v in W.items()}
    pred = ref.run(ir, graphs, torch.as_tensor(X, dtype=torch.float64), params)
    tr = torch.as_tensor(train)
    np.testing.assert_allclose(d["prediction"][train], pred[tr].detach().numpy(), rtol=1e-4, atol=1e-4)
    loss = torch.nn.functional.cross_entropy(pred[tr], torch.as_tensor(labels)[tr])
    np.testing.assert_allclose(d["losses"][0], loss.item(), rtol=1e-4, atol=1e-5)
    loss.backward()
    top = max(np.abs(p.grad.numpy()).max() for p in params.values())
    for k in W:
        want = params[name(k)].grad.numpy().reshape(-1)
        got = np.asarray(d["grad:" + k]).reshape(-1)
        tol = 1e-4 * np.abs(want).max() + 1e-6 * top
        assert np.abs(got - want).max() <= tol, (k, np.abs(got - want).max(), tol)

"""Programs emitted by the reference compiler's HIP generator, run on the MI355X.

refgen/build.py (run in the build container, where the reference's sources are) emits the
two-layer GCN (also kernel- and data-sampled), the three-layer GCN (also at config 5's layer
widths), GAT, GIN and GraphSAGE programs of
tests/dsl/<model>_ref_codegen.txt through
the reference's driver steps with HIPGenerator and compiles them over libgala_torch.so into
refgen/bin/.
Here each runs with GALA_DEVICE=cuda -- the base generator's model, autograd classes and
training loop, its aggregations and edge operators on libgala_hip.so's gfx950 kernels -- on a
20 000-row graph (the GAT one in 4 column tiles), and its first-epoch prediction, loss and
weight gradients are checked against galac's program of the same DSL in the float64 IR
executor (tests/_refgen_check.py; 1e-4). Nothing of the reference is read here.
"""
import os

import pytest

import _refgen_check as rc

BIN = os.path.join(rc.PKG, "refgen", "bin")


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("model", ["gcn", "gcn3", "gcn3_papers", "gcn_ksample", "gcn_dsample", "gat", "gat_unfused", "gin",
                                   "gin_motion", "sage", "gcn_train", "gcn3_train", "gat_train", "gin_train",
                                   "sage_train"])
def test_reference_emitted_program_on_the_gpu(tmp_path, model):
    """gat_unfused: the base's spelling of the GAT edge chain (its own autograd classes over the
    mirror's edge operators), gat: HIPGenerator's fused layer; both against galac's IR."""
    exe = os.path.join(BIN, "gala_" + model)
    if not os.path.exists(exe):
        pytest.skip(f"{exe} is not built (refgen/build.py needs the reference's sources)")
    feat, labels = (128, 172) if model == "gcn3_papers" else (64, 7)    # refgen/build.py's PROGRAMS
    d, X = rc.dataset(tmp_path, n=20000, nnz=240000, feat=feat, labels=labels, seed=11)
    # seeded weights (GALA_SEED): the same program run every time, so a miss reproduces
    dump = rc.run_program(exe, str(tmp_path), "cuda", seed=5)
    # 20 000 rows: the GAT attention-bias gradients' cancellation noise is ~5e-8 against a
    # 1.5e-2 largest gradient (the same on the host backend); the GCN-3 at config 5's widths
    # (128 / 128 / 172) sums its FFN weight gradients over the 20 000 rows in fp32 and has
    # measured up to 6e-5 of the model's largest gradient off on a weight whose own largest
    # entry is small (fc1: 7.4e-8 against 4.3e-4), hence a 1e-4 floor for that one tensor;
    # every other gradient keeps the 1e-5 floor
    rc.check_against_galac(model.replace("_unfused", ""), dump, d, X, tmp_path / "ir.json", noise_floor=1e-5,
                           floors={"fc1.weight": 1e-4} if model == "gcn3_papers" else None)


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("model", ["gcn3", "gcn3_papers", "gin", "sage", "gcn3_train"])
def test_fused_gcn_chains_bit_identical_to_the_base_spelling(tmp_path, model):
    """HIPGenerator's fused GCN chains (gcn_aggregate[_relu]_apply in place of the base's torch
    ROW_BROADCAST / ReLU ops around the aggregation, common.h:928-978,1150-1184) and its loss
    spelling (index_select + log_softmax / gather / mean for boolean indexing +
    CrossEntropyLoss): the first epoch's prediction and every weight gradient equal the
    unfused program's (GALA_REFGEN_UNFUSED) bit for bit; the loss is the same sum in another
    order."""
    import numpy as np
    exe, exe0 = (os.path.join(BIN, "gala_" + m) for m in (model, model + "_unfused"))
    if not (os.path.exists(exe) and os.path.exists(exe0)):
        pytest.skip("refgen programs not built (refgen/build.py needs the reference's sources)")
    feat, labels = (128, 172) if model == "gcn3_papers" else (64, 7)
    rc.dataset(tmp_path, n=20000, nnz=240000, feat=feat, labels=labels, seed=11)
    d1 = rc.run_program(exe, str(tmp_path), "cuda", seed=7)
    d0 = rc.run_program(exe0, str(tmp_path), "cuda", seed=7)
    assert set(d1) == set(d0)
    for k in d0:
        if k == "loss":
            np.testing.assert_allclose(d1[k], d0[k], rtol=1e-6, atol=0)
        else:
            np.testing.assert_array_equal(d1[k], d0[k], err_msg=k)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_fused_gat_chain_against_the_base_spelling(tmp_path):
    """HIPGenerator's fused GAT layer (gat_aggregate[_ffn]_apply in place of the base's edge sum,
    LeakyReLU, softmax and attention-weighted aggregation classes, common.h:622-894) beside the
    base's spelling over the mirror's K5 / K7 / K8 / K9 operators (GALA_REFGEN_UNFUSED), same
    seed: the fused kernels sum each row in the chain's order but round alpha = p * q once per
    edge where the chain stores it, so the first epoch's prediction, loss and weight gradients
    agree to fp32 rounding (1e-5 relative to each tensor's largest entry), not bit for bit."""
    import numpy as np
    exe, exe0 = (os.path.join(BIN, "gala_" + m) for m in ("gat", "gat_unfused"))
    if not (os.path.exists(exe) and os.path.exists(exe0)):
        pytest.skip("refgen programs not built (refgen/build.py needs the reference's sources)")
    rc.dataset(tmp_path, n=20000, nnz=240000, feat=64, labels=7, seed=11)
    d1 = rc.run_program(exe, str(tmp_path), "cuda", seed=7)
    d0 = rc.run_program(exe0, str(tmp_path), "cuda", seed=7)
    assert set(d1) == set(d0)
    top = max(np.abs(v).max() for k, v in d0.items() if k.endswith(".grad"))
    for k in d0:
        scale = np.abs(d0[k]).max()
        # gradients: 1e-5 of the tensor's largest entry plus 1e-6 of the model's (the attention
        # biases' gradients are cancellation noise, see tests/_refgen_check.py)
        tol = 1e-5 * scale + (1e-6 * top if k.endswith(".grad") else 0)
        assert np.abs(d1[k] - d0[k]).max() <= tol, (k, np.abs(d1[k] - d0[k]).max(), tol)

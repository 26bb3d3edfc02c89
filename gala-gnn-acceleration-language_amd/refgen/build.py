"""Build recipe of the reference-side HIP code generator's programs.

The reference compiler's driver steps with HIPGenerator (refgen/ir_driver.cpp, compiled
against the reference's own headers where they lie) emit a CMakeLists.txt + gala.cu; the
gala.cu is host C++ over the operator mirror (libgala_torch.so), compiled here with g++
against the reference's host headers. Needs /root/reference (or GALA_REF_ROOT); the GPU box
only runs the programs built here (refgen/bin/, git-ignored, shipped with the tree).

    python refgen/build.py            # refgen/bin/gala_{gcn,gcn3,gcn_ksample,gcn_dsample,gat,gin,gin_motion,sage}
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
REF = os.environ.get("GALA_REF_ROOT", "/root/reference")
BIN = os.path.join(HERE, "bin")

# the programs the GPU test runs: driver arguments after DATASET
# (FEAT LABELS HIDDEN ITERS COARSEN [COL_TILE]); the GAT one over 4 column tiles of 20 000 rows
PROGRAMS = {
    "gcn": ["64", "7", "32", "3", "2"],
    # three layers (config 5's GCN-3) over 4 column tiles of 20 000 rows
    "gcn3": ["64", "7", "32", "3", "2", "5000"],
    # config 5's GCN-3 at its own sizes (F 128, hidden 128, 172 labels, col_tile(1000000),
    # 10 epochs: bench/dsl/gcn3_papers10.txt), for tools/refgen_config5.py
    "gcn3_papers": ["128", "172", "128", "10", "2", "1000000"],
    # the kernel-sampled GCN of tests/GALA-DSL/ablations/sampling/kernel: sample(5), one tile
    "gcn_ksample": ["64", "7", "32", "3", "2", "10000000", "5"],
    # the data-sampled GCN of tests/GALA-DSL/ablations/sampling/data: G.sample(3), one tile
    "gcn_dsample": ["64", "7", "32", "3", "2", "10000000", "0", "3"],
    "gat": ["64", "7", "32", "3", "2", "5000"],
    # config 3's single-head drop-in shape (tests/GALA-DSL/gat/Products/h100.txt: F 100, hidden 32,
    # 47 labels, col_tile(10000000)), 10 epochs, for tools/refgen_gat_products.py
    "gat_products": ["100", "47", "32", "10", "2", "10000000"],
    "gin": ["64", "7", "32", "3", "2"],
    "gin_motion": ["64", "7", "32", "3", "2"],
    "sage": ["64", "7", "32", "3", "2"],
    # the GCN-3 programs without HIPGenerator's fused GCN chains and loss (GALA_REFGEN_UNFUSED):
    # the fused ones must give the same prediction and gradients bit for bit
    "gcn3_unfused": ["64", "7", "32", "3", "2", "5000"],
    "gcn3_papers_unfused": ["128", "172", "128", "10", "2", "1000000"],
    # the GAT program in the base's spelling: its own edge-sum / softmax / aggregation classes
    # over the mirror's K5 / K7 / K8 / K9 and weighted SpMM (the operator-level drop-in path)
    "gat_unfused": ["64", "7", "32", "3", "2", "5000"],
    # gala_train's whole pass set (GALA_REFGEN_TRAIN: reordering, sparse rewrites, code motion and
    # the training subgraph, tests/gala_train.cpp:124-146), the schedule of the paper's evaluation
    # (scripts/Evaluations/Figures-16-17.py:82): the GCN untiled and the GCN-3 over 4 column tiles
    # (the subgraphs' own tiled copies)
    "gcn_train": ["64", "7", "32", "3", "2"],
    "gcn3_train": ["64", "7", "32", "3", "2", "5000"],
    "gat_train": ["64", "7", "32", "3", "2", "5000"],
    "gin_train": ["64", "7", "32", "3", "2"],
    "sage_train": ["64", "7", "32", "3", "2"],
    # the base's spelling of the GIN, SAGE and gala_train GCN-3 programs (no fused chains, the
    # base's loss): the fused ones give the same prediction and gradients bit for bit
    "gin_unfused": ["64", "7", "32", "3", "2"],
    "sage_unfused": ["64", "7", "32", "3", "2"],
    "gcn3_train_unfused": ["64", "7", "32", "3", "2", "5000"],
}


def have_reference() -> bool:
    return os.path.isfile(os.path.join(REF, "src", "codegen", "common.h"))


def compile_driver(exe: str) -> None:
    subprocess.run(["g++", "-std=c++17", "-O1", "-w", f"-I{REF}", f"-I{REF}/src/codegen", f"-I{HERE}",
                    os.path.join(HERE, "ir_driver.cpp"), "-o", exe], check=True, capture_output=True, text=True,
                   timeout=300)


# gala_train's training-invariant code motion (tests/gala_train.cpp:136-140): for SAGE (without
# it the reference generator's first SAGE FFN reads t_iden_n, which only the hoisted mean
# aggregation defines, common.h:1210-1213) and for the GIN under gala_train's passes
CODE_MOTION = {"sage", "gin_motion", "sage_unfused"}


def emit(driver: str, out_dir: str, model: str, dataset: str, args) -> str:
    """Emit the program of `model` (a program name: gcn, gcn3, gcn_ksample, gcn_dsample, gat, gin, gin_motion,
    sage)."""
    os.makedirs(out_dir, exist_ok=True)
    env = dict(os.environ)
    if model in CODE_MOTION:
        env["GALA_REFGEN_CODE_MOTION"] = "1"
    if model.endswith("_unfused"):
        env["GALA_REFGEN_UNFUSED"] = "1"
    if "_train" in model:
        env["GALA_REFGEN_TRAIN"] = "1"
    family = model.split("_")[0]          # the driver's layer template (gcn3_papers: gcn3)
    subprocess.run([driver, out_dir.rstrip("/") + "/", family, dataset, *args], check=True, capture_output=True,
                   text=True, timeout=60, env=env)
    return os.path.join(out_dir, "gala.cu")


def compile_program(src: str, exe: str) -> None:
    import torch
    T = os.path.dirname(torch.__file__)
    subprocess.run(["g++", "-O2", "-std=c++17", "-w", "-fopenmp", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                    "-x", "c++", src, f"-I{REF}", f"-I{T}/include", f"-I{T}/include/torch/csrc/api/include",
                    "-I/opt/rocm/include", f"-I{PKG}/host", f"-I{ROOT}/include", "-o", exe, f"-L{T}/lib",
                    f"-Wl,-rpath,{T}/lib", "-Wl,--no-as-needed", "-ltorch", "-ltorch_cpu", "-lc10", "-lc10_hip",
                    "-ltorch_hip", f"-L{PKG}/gala", f"-Wl,-rpath,{PKG}/gala", "-lgala_torch", "-Wl,--as-needed"],
                   check=True, capture_output=True, text=True, timeout=600)


def build_all() -> None:
    os.makedirs(BIN, exist_ok=True)
    from concurrent.futures import ThreadPoolExecutor
    driver = os.path.join(BIN, "ir_driver")
    compile_driver(driver)
    srcs = {m: emit(driver, os.path.join(BIN, "src_" + m), m, "Cora", a) for m, a in PROGRAMS.items()}
    with ThreadPoolExecutor(max_workers=min(4, os.cpu_count() or 1)) as ex:   # g++ per program
        for m in ex.map(lambda m: (compile_program(srcs[m], os.path.join(BIN, "gala_" + m)), m)[1], srcs):
            print(f"refgen: built {os.path.join(BIN, 'gala_' + m)}")


if __name__ == "__main__":
    if not have_reference():
        print(f"refgen: {REF} is absent, nothing built", file=sys.stderr)
        sys.exit(0)
    build_all()

"""gala — MI355X (gfx950) hot path of GALA's generated GNN programs.

  gala._abi    ctypes mirror of include/gala_hip.h (libgala_hip.so)
  gala.layout  host graph layout builders (CSR build, column tiling, sampling)
  gala.ops     torch-facing functional ops on device tensors
  gala.torch_ext  (optional) the C++/libtorch mirror of the emitted operator API
"""
from . import _abi, layout  # noqa: F401

__all__ = ["_abi", "layout", "torch_ext"]


def torch_ext():
    """The C++/libtorch operator mirror (host/gala_torch.cpp) as a Python module."""
    import torch  # noqa: F401  (loads libtorch before the extension)
    from . import _gala_torch
    return _gala_torch

"""torch_distlearn_amd -- an MI355X-native (gfx950, PyTorch-ROCm + HIP + RCCL)
data-parallel training library with the capabilities and API of
shanlior/torch-distlearn:

* ``AllReduceSGD(tree)``            synchronous DP with uneven-step handling
* ``AllReduceEA(tree, tau, alpha)`` synchronous elastic averaging
* ``AsyncEA(...)``                  asynchronous EASGD parameter server
* ``Tree`` / ``LocalhostTree``      the collective object (RCCL data plane, gloo control)
* ``printServer`` / ``printClient`` coloured protocol logging
"""
import torch  # noqa: F401  (load torch's HIP runtime + RCCL before the native library)

from .parallel import (AllReduceEA, AllReduceSGD, AsyncEA, Communicator, FlatBuffer, GradBucketer, LocalhostTree,
                       Tree, init_communicator)
from .ops.flat import FlatParams
from .utils.color_print import printClient, printServer
from .utils.walk import walkTable, walk_table
from . import _native

__version__ = "0.1.0"

__all__ = ["AllReduceSGD", "AllReduceEA", "AsyncEA", "Tree", "LocalhostTree", "Communicator", "FlatBuffer",
           "FlatParams", "GradBucketer", "init_communicator", "printServer", "printClient", "walkTable",
           "walk_table"]

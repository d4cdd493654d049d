"""Data-parallel algorithms and the collective layer."""
from .comm import Communicator, ProcessGroupCommunicator, RcclCommunicator, init_communicator
from .tree import FlatBuffer, LocalhostTree, Tree
from .buckets import GradBucketer
from .allreduce_sgd import AllReduceSGD
from .allreduce_ea import AllReduceEA
from .async_ea import AsyncEA

__all__ = ["Communicator", "ProcessGroupCommunicator", "RcclCommunicator", "init_communicator", "FlatBuffer",
           "LocalhostTree", "Tree", "GradBucketer", "AllReduceSGD", "AllReduceEA", "AsyncEA"]

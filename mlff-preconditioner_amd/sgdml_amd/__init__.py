"""sgdml_amd — MI355X (gfx950) preconditioned-CG solver for the sGDML kernel system.

Drop-in replacement of the solve path of bluecher31/mlff-preconditioner:
`sgdml_amd.solvers.iterative_solver.Iterative` mirrors the reference's
`sgdml.solvers.iterative_solver.Iterative` (iterative_solver.py:75-1108); the
numerics run in libmlffpcg.so (hand-written HIP kernels, include/mlffpcg.h).
"""
from ._native import load_library, device_count, comm_unique_id  # noqa: F401
from .solver import KernelSolver, PCGResult, host_descriptors, sgdml_descriptors  # noqa: F401
from .sharded import ShardedKernelSolver  # noqa: F401
from .rule_of_thumb import get_params, rule_of_thumb  # noqa: F401

__version__ = "0.1.0"
from . import synthetic  # noqa: F401,E402

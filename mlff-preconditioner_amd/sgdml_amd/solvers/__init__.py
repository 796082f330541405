"""Solvers with the reference's interface (sgdml.solvers)."""
from .iterative_solver import Iterative  # noqa: F401

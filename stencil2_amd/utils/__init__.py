"""Utilities: statistics, ParaView CSV reader, weak-scaling helpers."""
from .paraview import read_paraview  # noqa: F401
from .stats import summarize  # noqa: F401

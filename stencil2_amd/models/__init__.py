"""Stencil applications (the reference's bin/jacobi3d.cu and bin/astaroth_sim.cu) as models."""
from .stencil_model import Jacobi3D, AstarothSim, StencilModel, weak_scaled_size  # noqa: F401

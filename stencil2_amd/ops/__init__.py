"""Kernel entry points and pure-torch fp32/fp64 oracles (used by the numerics tests)."""
from .reference import (  # noqa: F401
    astaroth_init_reference,
    astaroth_step_reference,
    jacobi_spheres,
    jacobi_step_reference,
    periodic_gather,
)
from .kernels import stencil7_apply, stencil7x2_apply, stencil7x2_supported  # noqa: F401

"""Thin wrappers over the native HIP kernels (csrc/src/kernels/*.hip)."""
from __future__ import annotations

from .. import _C


def stencil7_apply(dd, di: int, q: int, region, kind=_C.StencilKind.Jacobi, spheres: bool = True, stream: int = 0):
    """next(region) = 7-point stencil of curr for quantity q of local sub-domain di (HIP kernel on its GPU)."""
    native = getattr(dd, "native", dd)
    _C.stencil7_apply(native, di, q, region, kind, spheres, stream)

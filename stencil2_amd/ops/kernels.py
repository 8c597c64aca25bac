"""Thin wrappers over the native HIP kernels (csrc/src/kernels/*.hip)."""
from __future__ import annotations

from .. import _C


def stencil7_apply(dd, di: int, q: int, region, kind=_C.StencilKind.Jacobi, spheres: bool = True, stream: int = 0):
    """next(region) = 7-point stencil of curr for quantity q of local sub-domain di (HIP kernel on its GPU)."""
    native = getattr(dd, "native", dd)
    _C.stencil7_apply(native, di, q, region, kind, spheres, stream)


def stencil7x2_supported(dd, di: int, q: int) -> bool:
    """True when the fused two-step kernel can run on quantity q of local sub-domain di: a device fp32/fp64 quantity,
    face radii >= 2 (edges >= 1) and the aligned row layout."""
    return _C.stencil7x2_supported(getattr(dd, "native", dd), di, q)


def stencil7x2_apply(dd, di: int, q: int, region, kind=_C.StencilKind.Jacobi, spheres: bool = True, stream: int = 0,
                     tune=None):
    """next(region) = S(S(curr)) -- two fused 7-point steps (temporal blocking), bitwise equal to two single steps --
    for quantity q of local sub-domain di. The depth-2 face and depth-1 edge halos of curr must be valid (exchange()
    first); with `tune.wrap` set, the axes in that mask are read periodically in-kernel instead (the region must then
    span them). One read and one write of the field per two steps (csrc/src/kernels/stencil7x2.hip)."""
    native = getattr(dd, "native", dd)
    _C.stencil7x2_apply(native, di, q, region, kind, spheres, stream, tune if tune is not None else _C.StencilTune())

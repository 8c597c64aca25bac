"""Pure-torch references of the runtime's semantics (periodic halos, Jacobi3D, Astaroth proxy).

The operation order matches the reference CUDA kernels (bin/jacobi3d.cu:72-83: +x,-x,+y,-y,+z,-z then /6;
bin/astaroth_sim.cu:72-81: -x,-y,-z,+x,+y,+z then /6), so fp32 results are expected to be bitwise equal to the HIP
kernels. Sphere membership uses the exact integer form of the reference's truncated float sqrt:
floor(sqrt(d2)) <= R  <=>  d2 < (R+1)^2.
"""
from __future__ import annotations

import math

import torch


def periodic_gather(g: torch.Tensor, origin, raw_size) -> torch.Tensor:
    """Values of the (z, y, x) global periodic grid `g` on the box starting at global `origin` (x, y, z)."""
    Z, Y, X = g.shape
    ox, oy, oz = origin
    rx, ry, rz = raw_size
    iz = (torch.arange(rz) + oz) % Z
    iy = (torch.arange(ry) + oy) % Y
    ix = (torch.arange(rx) + ox) % X
    return g[iz][:, iy][:, :, ix]


def jacobi_spheres(size):
    """(hot_xyz, cold_xyz, radius) for a global grid of `size` (x, y, z) (bin/jacobi3d.cu:45-50)."""
    X, Y, Z = size
    hot = (X // 3, Y // 2, Z // 2)
    cold = (X * 2 // 3, Y // 2, Z // 2)
    return hot, cold, X // 10


def _sphere_masks(shape_zyx, size_xyz, device):
    Z, Y, X = shape_zyx
    hot, cold, R = jacobi_spheres(size_xyz)
    z = torch.arange(Z, device=device).view(-1, 1, 1)
    y = torch.arange(Y, device=device).view(1, -1, 1)
    x = torch.arange(X, device=device).view(1, 1, -1)
    r1 = (R + 1) ** 2
    dh = (x - hot[0]) ** 2 + (y - hot[1]) ** 2 + (z - hot[2]) ** 2
    dc = (x - cold[0]) ** 2 + (y - cold[1]) ** 2 + (z - cold[2]) ** 2
    return dh < r1, dc < r1


def _div6(val: torch.Tensor) -> torch.Tensor:
    """IEEE val / 6 on any device. PyTorch's GPU kernel turns a division by a Python / CPU scalar into a
    multiplication by its (rounded) reciprocal, which differs in the last bit; a divisor tensor on the same device
    keeps the true division the kernels implement."""
    if val.device.type == "cpu":
        return val / 6
    return val / torch.full((), 6, dtype=val.dtype, device=val.device)


def jacobi_step_reference(u: torch.Tensor) -> torch.Tensor:
    """One Jacobi3D iteration on a periodic global (z, y, x) grid."""
    Z, Y, X = u.shape
    px = torch.roll(u, -1, 2)
    mx = torch.roll(u, 1, 2)
    py = torch.roll(u, -1, 1)
    my = torch.roll(u, 1, 1)
    pz = torch.roll(u, -1, 0)
    mz = torch.roll(u, 1, 0)
    val = torch.zeros_like(u) + px  # leading 0 + as in the reference kernel (sign of zero)
    val = val + mx
    val = val + py
    val = val + my
    val = val + pz
    val = val + mz
    val = _div6(val)
    hot, cold = _sphere_masks(u.shape, (X, Y, Z), u.device)
    val = torch.where(hot, torch.ones_like(val), val)
    val = torch.where(cold & ~hot, torch.zeros_like(val), val)
    return val


def astaroth_step_reference(u: torch.Tensor) -> torch.Tensor:
    """One Astaroth-proxy iteration (6-neighbour mean) on a periodic global (z, y, x) grid."""
    mx = torch.roll(u, 1, 2)
    my = torch.roll(u, 1, 1)
    mz = torch.roll(u, 1, 0)
    px = torch.roll(u, -1, 2)
    py = torch.roll(u, -1, 1)
    pz = torch.roll(u, -1, 0)
    val = torch.zeros_like(u) + mx
    val = val + my
    val = val + mz
    val = val + px
    val = val + py
    val = val + pz
    return _div6(val)


def astaroth_init_reference(size_xyz, radius: int, period: float, dtype=torch.float32) -> torch.Tensor:
    """Global interior initial condition of the Astaroth proxy: sin(2*pi'/period*(g+r)) summed over axes, where
    pi' = 3.14159 and (g + r) is the raw allocation index of the owning sub-domain (bin/astaroth_sim.cu:50-53)."""
    X, Y, Z = size_xyz
    k = 2 * 3.14159 / period
    z = torch.arange(Z, dtype=torch.float64).view(-1, 1, 1) + radius
    y = torch.arange(Y, dtype=torch.float64).view(1, -1, 1) + radius
    x = torch.arange(X, dtype=torch.float64).view(1, 1, -1) + radius
    return torch.sin(k * x + k * y + k * z).to(dtype)


__all__ = ["periodic_gather", "jacobi_spheres", "jacobi_step_reference", "astaroth_step_reference",
           "astaroth_init_reference", "math"]

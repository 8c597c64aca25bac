"""Analytic exchange oracles shared by the tests and the GPU validation scripts.

Same idea as the reference's tests (test/test_exchange.cu:12-38 "ripple", test_cuda_mpi_distributed_domain.cu:10-22
coordinate packing): every interior cell holds a function of its global coordinate; after exchange() every halo
cell in direction d must hold the value at its periodic image iff radius(d) != 0, and keep its poison otherwise.
"""
from __future__ import annotations

import torch

POISON = -1


def encode(gz, gy, gx):
    return gx + 1000 * gy + 1000000 * gz


def fill_coords(dd, q: int, poison: int = POISON, offset: int = 0):
    """Poison whole allocations (curr and next), then write encode(global coord) + offset into every interior cell."""
    for di in range(dd.num_domains()):
        for curr in (True, False):
            t = dd.curr(di, q) if curr else dd.next(di, q)
            t.fill_(poison)
    dd.fill_from_global(q, lambda z, y, x: encode(z, y, x) + offset)


def expected_full(dd, di: int, radius, poison: int = POISON, boundary=None, offset: int = 0) -> torch.Tensor:
    d = dd.domain(di)
    org, raw, sz = d.accessor_origin(), d.raw_size(), d.size()
    cr = d.get_compute_region()
    Z, Y, X = dd.size().z, dd.size().y, dd.size().x
    gz = torch.arange(raw.z).view(-1, 1, 1) + org.z
    gy = torch.arange(raw.y).view(1, -1, 1) + org.y
    gx = torch.arange(raw.x).view(1, 1, -1) + org.x
    dz = (gz >= cr.hi.z).long() - (gz < cr.lo.z).long()
    dy = (gy >= cr.hi.y).long() - (gy < cr.lo.y).long()
    dx = (gx >= cr.hi.x).long() - (gx < cr.lo.x).long()
    dz, dy, dx = torch.broadcast_tensors(dz, dy, dx)
    want = (encode(gz % Z, gy % Y, gx % X) + offset).expand(raw.z, raw.y, raw.x).clone()
    filled = torch.zeros_like(want, dtype=torch.bool)
    for zz in (-1, 0, 1):
        for yy in (-1, 0, 1):
            for xx in (-1, 0, 1):
                sel = (dz == zz) & (dy == yy) & (dx == xx)
                if (xx, yy, zz) == (0, 0, 0) or radius.dir(xx, yy, zz) != 0:
                    filled |= sel
    if boundary is not None:
        # nothing crosses a non-periodic face of the global grid: cells outside it keep their poison
        for axis, (g, n) in enumerate(((gx, X), (gy, Y), (gz, Z))):
            for side in (-1, 1):
                face = [0, 0, 0]
                face[axis] = side
                if not boundary.face_periodic(*face):
                    out = (g < 0) if side < 0 else (g >= n)
                    filled &= ~out.expand_as(filled)
    want[~filled] = poison
    return want


def check_exchange(dd, q: int, radius, poison: int = POISON, boundary=None, offset: int = 0):
    """Return the number of wrong cells over every local sub-domain."""
    bad = 0
    for di in range(dd.num_domains()):
        t = dd.curr(di, q).cpu()
        if t.is_floating_point():
            # NaN poison (race canary) must never survive in a cell that should have been written
            t = torch.nan_to_num(t, nan=float(poison))
        got = t.long()
        want = expected_full(dd, di, radius, poison, boundary, offset)
        bad += int((got != want).sum())
    return bad

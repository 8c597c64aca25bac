"""Python face of the native DistributedDomain, with zero-copy torch views of every quantity.

Parity: reference include/stencil/stencil.hpp (DistributedDomain API). The views are DLPack exports of the
runtime's halo-padded allocations: ``curr(di, q)`` has shape (z, y, x) = raw_size (interior + halo) and the padded
x pitch as its stride, so writes through the tensor are seen by the HIP kernels and vice versa.
"""
from __future__ import annotations

import torch

from .. import _C
from .process_group import get_group

_TORCH_TO_DT = {
    torch.float32: _C.DType.F32,
    torch.float64: _C.DType.F64,
    torch.int32: _C.DType.I32,
    torch.int64: _C.DType.I64,
    torch.uint8: _C.DType.U8,
    torch.int8: _C.DType.I8,
    torch.float16: _C.DType.F16,
    torch.bfloat16: _C.DType.BF16,
}


class DistributedDomain:
    """A periodic global grid split into sub-domains (one per GPU, several per process allowed)."""

    def __init__(self, x: int, y: int, z: int, group=None):
        self._group = group if group is not None else get_group()
        self._dd = _C.DistributedDomain(int(x), int(y), int(z), self._group)
        self._dtypes: list[torch.dtype] = []

    # -------- configuration --------
    def set_radius(self, r):
        self._dd.set_radius(r)

    def add_data(self, name: str = "", dtype: torch.dtype = torch.float32) -> int:
        """Register a quantity; returns its index (the reference's DataHandle)."""
        self._dtypes.append(dtype)
        es = torch.empty((), dtype=dtype).element_size()
        return self._dd.add_data(es, name, _TORCH_TO_DT.get(dtype, _C.DType.Bytes))

    def __getattr__(self, name):
        return getattr(self._dd, name)

    @property
    def native(self):
        return self._dd

    # -------- views --------
    def domains(self):
        return [self._dd.domain(i) for i in range(self._dd.num_domains())]

    def curr(self, di: int, q: int = 0) -> torch.Tensor:
        """(z, y, x) view of the whole allocation (halo included) of the current buffer."""
        return torch.from_dlpack(self._dd.dlpack(di, q, True))

    def next(self, di: int, q: int = 0) -> torch.Tensor:
        return torch.from_dlpack(self._dd.dlpack(di, q, False))

    def interior(self, t: torch.Tensor, di: int) -> torch.Tensor:
        """Slice the interior (compute region) out of a full view."""
        d = self._dd.domain(di)
        r = d.radius()
        sz = d.size()
        return t[r.z(-1): r.z(-1) + sz.z, r.y(-1): r.y(-1) + sz.y, r.x(-1): r.x(-1) + sz.x]

    def curr_interior(self, di: int, q: int = 0) -> torch.Tensor:
        return self.interior(self.curr(di, q), di)

    def origin(self, di: int):
        return self._dd.get_origin(di)

    def fill_from_global(self, q: int, fn, include_halo: bool = False):
        """Set every local cell of quantity q to fn(gz, gy, gx) (torch index tensors of global coordinates)."""
        for di, d in enumerate(self.domains()):
            t = self.curr(di, q)
            org = d.accessor_origin()
            raw = d.raw_size()
            dev = t.device
            gz = torch.arange(raw.z, device=dev).view(-1, 1, 1) + org.z
            gy = torch.arange(raw.y, device=dev).view(1, -1, 1) + org.y
            gx = torch.arange(raw.x, device=dev).view(1, 1, -1) + org.x
            vals = fn(gz, gy, gx).to(t.dtype)
            if include_halo:
                t.copy_(vals.expand_as(t))
            else:
                self.interior(t, di).copy_(self.interior(vals.expand(raw.z, raw.y, raw.x), di))
        if torch.cuda.is_available():
            torch.cuda.synchronize()

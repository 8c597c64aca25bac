"""Jacobi3D / Astaroth proxy models on the native StencilModel (csrc/src/stencil_model.cpp).

Each ``step()`` enqueues interior compute, the halo exchange and the exterior compute on HIP streams without any
host synchronisation (see csrc/include/stencil/models/stencil_model.hpp); ``synchronize()`` waits.
Reference: bin/jacobi3d.cu (weak scaling, hot/cold spheres), bin/astaroth_sim.cu (radius 3, 26 directions).
"""
from __future__ import annotations

import torch

from .. import _C
from ..parallel.process_group import get_group


def weak_scaled_size(per_gpu: int, n: int) -> int:
    """Reference weak-scaling rule: each axis = per_gpu * n**0.33333, rounded (bin/jacobi3d.cu:167-169)."""
    return int(per_gpu * float(n) ** 0.33333 + 0.5)


class StencilModel:
    def __init__(self, size, kind=_C.StencilKind.Jacobi, radius: int = 1, all_directions: bool = False,
                 quantities: int = 1, fp64: bool = False, methods=_C.MethodFlags.All,
                 placement=_C.PlacementStrategy.NodeAware, gpus=None, overlap: bool = True, auto_overlap: bool = True,
                 use_graph: bool = True, forward: bool = False, temporal: int = 1, backend=None,
                 tune: _C.StencilTune | None = None, group=None, axis_cost=None, wrap_self: bool = True,
                 transport: _C.TransportOptions | None = None, wrap_axes_mask: int = 7, local_interior: bool = True,
                 overlap_mode: int = 1, self_test: bool = False, partition=None, x_halo_align: bool = False,
                 interior_align: int = 128, row_pad_lines: int = 0, shared_halo_line: bool = False):
        cfg = _C.StencilModelConfig()
        cfg.size = _C.Dim3(*size)
        cfg.kind = kind
        cfg.radius = radius
        cfg.all_directions = all_directions
        cfg.quantities = quantities
        cfg.fp64 = fp64
        cfg.methods = methods
        cfg.placement = placement
        if gpus is not None:
            cfg.gpus = list(gpus)
        cfg.overlap = overlap
        cfg.auto_overlap = auto_overlap
        cfg.use_graph = use_graph
        cfg.forward = forward
        cfg.temporal = temporal
        cfg.wrap_self = wrap_self
        cfg.wrap_axes_mask = wrap_axes_mask
        cfg.local_interior = local_interior
        cfg.overlap_mode = overlap_mode
        cfg.self_test = self_test  # multi-rank: verify the transports on a probe domain, ladder to what works
        cfg.x_halo_align = x_halo_align  # x halos inside the interior's first / last 64-B sector
        cfg.interior_align = interior_align  # byte alignment of every row's first interior cell (128 or 64)
        cfg.row_pad_lines = row_pad_lines  # extra 128-B lines per row pitch (measurement knob)
        cfg.shared_halo_line = shared_halo_line  # row r's +x and row r+1's -x halo in one 128-B line
        if transport is not None:  # DistributedDomain.set_transport_options (inbox memory, DMA copies, completion)
            cfg.transport = transport
        if backend is not None:
            cfg.backend = backend
        if tune is not None:
            cfg.tune = tune
        if axis_cost is not None:  # NodeAware cut costs per axis (default (4, 3, 2): x faces are strided and
            # whole periodic rows feed the whole-row kernels; z cuts before y cuts)
            cfg.axis_cost = _C.Dim3(*axis_cost)
        if partition is not None:  # NodeAware cut rule inside a node: PartitionObjective.Interface (reference) or
            cfg.partition = partition  # MaxLink (busiest xGMI link, then total halo)
        self.config = cfg
        self._m = _C.StencilModel(cfg, group if group is not None else get_group())
        self._dd = None

    def init(self):
        self._m.init()
        self._dd = self._m.domain()
        return self

    def step(self):
        self._m.step()

    def run(self, iters: int):
        self._m.run(iters)

    def prepare(self, runs=()):
        """Instantiate run()'s hipGraph blocks for both buffer parities (records work, runs nothing); for each length n
        in `runs` also a graph of a whole run(n), which run(n) then replays as one launch."""
        self._m.prepare(list(runs))

    def synchronize(self):
        self._m.synchronize()

    @property
    def domain(self):
        return self._dd

    def overlapping(self) -> bool:
        return self._m.overlapping()

    def can_toggle_overlap(self) -> bool:
        """True when the fused pairs have remote halos and can run overlapped or whole-region (set_overlap)."""
        return self._m.can_toggle_overlap()

    def set_overlap(self, on: bool):
        """Switch fused pairs between overlapped (local interior during the transfers, slabs after) and whole-region
        (exchange, then one sweep); synchronizes first."""
        self._m.set_overlap(bool(on))

    def set_overlap_mode(self, mode: int):
        """0 = whole-region pairs; 1 = overlapped, slabs on the comm stream beside the interior sweep; 2 = overlapped,
        slabs after the interior sweep on the compute stream; 3 = pipelined (can_pipeline()): whole-region sweeps that
        publish their boundary z planes, the next pair's exchange gated on them runs beside the rest of the sweep."""
        self._m.set_overlap_mode(int(mode))

    def can_pipeline(self) -> bool:
        """Overlap mode 3 is possible: one device, remote halos along z only, whole-row kernel, fused IPC stores."""
        return self._m.can_pipeline()

    def can_pipeline_triples(self) -> bool:
        """True when overlap mode 4 is possible: fused triples whose boundary z planes gate the next depth-3 exchange."""
        return self._m.can_pipeline_triples()

    def overlap_mode(self) -> int:
        return self._m.overlap_mode()

    def set_comm_reserve(self, cus: int):
        """CUs the overlapped sweeps leave to the transport kernels (StencilTune.x2reserve)."""
        self._m.set_comm_reserve(int(cus))

    def set_triple_schedule(self, sphw: float, left: int, parts: int = 0):
        """The fused triples' lockstep schedule (StencilTune x3sphw / x3left / x3parts; results are bitwise the same).
        Synchronizes and drops the recorded hipGraphs: prepare() again before a timed loop."""
        self._m.set_triple_schedule(float(sphw), int(left), int(parts))

    def comm_reserve(self) -> int:
        return self._m.comm_reserve()

    def local_interior_steps(self) -> bool:
        """True when overlapped single steps sweep the local interior (shrunk only at remote faces) during the
        remote transfers and wrap the self-periodic axes in-kernel."""
        return self._m.local_interior_steps()

    def temporal_blocking(self) -> bool:
        """True when run() advances in fused pairs of steps (stencil7x2, one depth-2 exchange per pair)."""
        return self._m.temporal_blocking()

    def temporal_triples(self) -> bool:
        """True when run() advances in fused triples of steps (stencil7x3, temporal=3 on one fully periodic GPU)."""
        return self._m.temporal_triples()

    def wrap_axes(self) -> int:
        """Axes (mask 1=x, 2=y, 4=z) the fused pairs read periodically in-kernel instead of from copied halos."""
        return self._m.wrap_axes()

    def step_wrap_axes(self) -> int:
        """Axes single steps read periodically in-kernel instead of from copied halos (0 = every halo copied)."""
        return self._m.step_wrap_axes()

    def forwarding(self) -> bool:
        """True when the stencil kernels write the neighbours' halos directly (in-process exchanges only)."""
        return self._m.forwarding()

    def cells(self) -> int:
        return self._m.cells()

    def local_cells(self) -> int:
        return self._m.local_cells()

    def field(self, di: int = 0, q: int = 0, curr: bool = True) -> torch.Tensor:
        """Full (z, y, x) view including halo."""
        return torch.from_dlpack(self._dd.dlpack(di, q, curr))

    def interior(self, di: int = 0, q: int = 0) -> torch.Tensor:
        d = self._dd.domain(di)
        r, sz = d.radius(), d.size()
        t = self.field(di, q)
        return t[r.z(-1): r.z(-1) + sz.z, r.y(-1): r.y(-1) + sz.y, r.x(-1): r.x(-1) + sz.x]


class Jacobi3D(StencilModel):
    def __init__(self, size=(512, 512, 512), **kw):
        super().__init__(size, kind=_C.StencilKind.Jacobi, radius=1, all_directions=False, **kw)


class AstarothSim(StencilModel):
    def __init__(self, size=(512, 512, 512), quantities: int = 8, **kw):
        super().__init__(size, kind=_C.StencilKind.Astaroth, radius=3, all_directions=True, quantities=quantities,
                         **kw)

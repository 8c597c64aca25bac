"""stencil2_amd — an MI355X-native 3D stencil halo-exchange runtime.

Capabilities of mengshanfeng/stencil-2 (DistributedDomain / LocalDomain / Radius / placement / transports /
ParaView output / Jacobi3D and Astaroth apps), re-designed for CDNA4 (gfx950): hand-written HIP kernels, HIP IPC
and RCCL over xGMI, one process per GPU or several GPUs per process.

Layout:
    stencil2_amd._C        native runtime (C++/HIP, csrc/), pybind11 bindings
    stencil2_amd.parallel  process groups, DistributedDomain with torch tensor views, placement helpers
    stencil2_amd.models    Jacobi3D / Astaroth proxy models (stream-ordered, overlapped exchange)
    stencil2_amd.ops       kernel entry points + pure-torch fp32 oracles used by the tests
    stencil2_amd.utils     statistics, weak-scaling sizes, ParaView CSV reader
"""
from __future__ import annotations

import os as _os

# torch must be imported before the native module: torch ships its own libamdhip64/librccl and the runtime must
# bind to those (same SONAME) instead of loading a second HIP runtime from /opt/rocm.
import torch as _torch  # noqa: F401

from . import _build

if _os.environ.get("STENCIL_SKIP_BUILD") != "1":
    _build.ensure_built()

from . import _C  # noqa: E402
from ._C import (  # noqa: E402,F401
    Backend,
    Boundary,
    Dim3,
    DType,
    MethodFlags,
    NodeAwarePlacement,
    NodePartition,
    PartitionObjective,
    PlacementStrategy,
    Radius,
    RankPartition,
    Rect3,
    Statistics,
    StencilError,
    StencilKind,
    StencilModelConfig,
    StencilTune,
    TransportOptions,
    TrivialPlacement,
    build_info,
    build_info_string,
    device_count,
    find_free_port,
    gpu_bandwidth,
    gpu_distance,
    gpu_links,
    halo_volume,
    make_reciprocal,
    make_single_group,
    make_tcp_group,
    methods_to_string,
    prime_factors,
    qap_cost,
    qap_solve,
    qap_solve_catch,
)
from .parallel.process_group import init_process_group, get_group  # noqa: E402,F401
from .parallel.domain import DistributedDomain  # noqa: E402,F401
from .models.stencil_model import Jacobi3D, AstarothSim, StencilModel  # noqa: E402,F401

__all__ = [
    "Backend", "Boundary", "Dim3", "DType", "MethodFlags", "PlacementStrategy", "Radius", "Rect3", "Statistics", "StencilKind",
    "DistributedDomain", "Jacobi3D", "AstarothSim", "StencilModel", "init_process_group", "get_group",
    "TransportOptions", "build_info", "RankPartition", "NodePartition", "TrivialPlacement", "NodeAwarePlacement", "qap_solve", "qap_solve_catch",
]

"""Process-group bootstrap for the native runtime.

The runtime's control plane (placement all-gathers, IPC handle exchange, host-staged fallback) runs on a native
TCP full mesh (csrc/src/proc_group.cpp) — the reference used MPI for this. When torch.distributed is
initialised (e.g. under torchrun), rank 0 picks a free port and publishes it through torch's store, so no extra
port has to be agreed on; otherwise RANK/WORLD_SIZE/MASTER_ADDR and MASTER_PORT+1 (or STENCIL_MASTER_PORT) are used.
"""
from __future__ import annotations

import os

from .. import _C

_group = None
_counter = 0


def _env_int(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v is not None:
            return int(v)
    return default


def init_process_group(rank: int | None = None, world_size: int | None = None, timeout_s: float = 600.0,
                       set_default: bool = True):
    """Create (or return) the native process group for this process."""
    global _group, _counter
    if _group is not None and rank is None and world_size is None:
        return _group
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        rank = dist.get_rank() if rank is None else rank
        world_size = dist.get_world_size() if world_size is None else world_size
        if world_size == 1:
            g = _C.make_single_group()
        else:
            store = dist.distributed_c10d._get_default_store()
            key = f"stencil2_amd/bootstrap/{_counter}"
            _counter += 1
            addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
            if rank == 0:
                port = _C.find_free_port()
                store.set(key, f"{addr}:{port}")
            val = store.get(key).decode()
            host, port = val.rsplit(":", 1)
            g = _C.make_tcp_group(rank, world_size, host, int(port), timeout_s)
    else:
        rank = _env_int("STENCIL_RANK", "RANK", default=0) if rank is None else rank
        world_size = _env_int("STENCIL_WORLD_SIZE", "WORLD_SIZE", default=1) if world_size is None else world_size
        if world_size == 1:
            g = _C.make_single_group()
        else:
            addr = os.environ.get("STENCIL_MASTER_ADDR", os.environ.get("MASTER_ADDR", "127.0.0.1"))
            port = _env_int("STENCIL_MASTER_PORT")
            if port is None:
                port = _env_int("MASTER_PORT", default=29500) + 1
            g = _C.make_tcp_group(rank, world_size, addr, port, timeout_s)
    if set_default:
        _C.set_default_group(g)
        _group = g
    return g


def get_group():
    return _group if _group is not None else init_process_group()

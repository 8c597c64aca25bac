"""Parallelism: process groups (native TCP bootstrap, torch.distributed rendezvous), DistributedDomain views."""
from .process_group import init_process_group, get_group  # noqa: F401
from .domain import DistributedDomain  # noqa: F401

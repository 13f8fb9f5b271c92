"""Sharded LBA windows over torch.distributed.

One process per GPU. Every rank holds the whole window (the caller's graph) and a plba
context bound to its GPU; the context keeps the landmarks of this rank's shard
(`plba_shard_plan`) and sums the partial reduced camera system with the other ranks once per
LM trial. Transports:

  rccl  the library's own RCCL communicator on the solver stream (captured into the step
        hipGraph). torch.distributed only carries the 128-byte RCCL unique id at setup.
  host  the library stages each all-reduce through pinned host memory and calls back into
        Python, which sums with torch.distributed (gloo). Used by tests that run several ranks
        on one GPU and on hosts without RCCL.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from .lib import Solver, comm_unique_id


def broadcast_unique_id(group=None) -> bytes:
    """Rank 0 creates the RCCL unique id; every rank returns the same 128 bytes."""
    import torch.distributed as dist
    obj = [comm_unique_id() if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return obj[0]


def host_allreduce(group=None):
    """In-place float64 sum over the ranks of `group` (gloo) for Solver.comm_init_host."""
    import torch
    import torch.distributed as dist

    def fn(buf: np.ndarray):
        t = torch.from_numpy(buf)      # shares memory with the pinned staging buffer
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return fn


def sharded_solver(device: int, transport: str = "rccl", group=None, rank: Optional[int] = None,
                   world: Optional[int] = None, **opts) -> Solver:
    """A Solver whose next upload() keeps this rank's shard of the window."""
    import torch.distributed as dist
    rank = dist.get_rank(group) if rank is None else rank
    world = dist.get_world_size(group) if world is None else world
    s = Solver(device=device, **opts)
    if transport == "rccl":
        s.comm_init_rccl(world, rank, broadcast_unique_id(group))
    elif transport == "host":
        s.comm_init_host(world, rank, host_allreduce(group))
    else:
        raise ValueError(f"unknown transport {transport!r}")
    return s


def comm_summary(infos: list) -> dict:
    """Summary of every rank's Solver.comm_info(): the rank counts RCCL reports, whether the ranks
    are 0..N-1 each once, and how many distinct devices (HIP ordinal + PCI location) they ran on."""
    n = len(infos)
    return {
        "ranks": infos,
        "rccl_ranks": sorted({int(c["ranks"]) for c in infos}),
        "rank_set_ok": sorted(int(c["rank"]) for c in infos) == list(range(n))
                       and all(int(c["ranks"]) == n for c in infos),
        "distinct_hip_devices": len({(c["hip_device"], c["pci"]) for c in infos}),
        "distinct_pci": len({c["pci"] for c in infos}),
    }


def gather_comm_info(info: dict, group=None) -> dict:
    """All ranks' comm_info() gathered on every rank (gloo object all-gather), summarised."""
    import torch.distributed as dist
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, info, group=group)
    return comm_summary(out)

"""Data-plane bootstrap of CPU runtimes through the replicated store.

On a GPU the data plane is the compiled DataPlane (csrc/core/dataplane.cpp,
``parallel.native_group``): RCCL over xGMI, or IpcComm, formed without any torch
process group.  A CPU runtime (tests, GPU-less hosts) runs the same pipeline
over a torch gloo group, formed the same way -- through the control plane the
members already share, no external launcher, no torchrun:

1. wait until ``world`` nodes of the service are registered (their 2 s leases
   are alive) -- the registry of cluster/registry.go:93-117;
2. the lowest node (sorted ``address:port``) opens a ``TCPStore`` and publishes
   ``{addr, port, members}`` under ``store/_ptype/nccl/<service>/<epoch>/<node>``;
   the record with the lowest create revision wins (``WithSort(SortByCreateRevision,
   SortAscend)``), so candidates with different views still converge;
3. every member initialises the gloo group from that store with
   ``rank = members.index(node)``.

``ElasticDataPlane`` (parallel/elastic.py) forms every later generation the
same way after a rank failure (epoch = generation).
"""
from __future__ import annotations

import json
import time
from datetime import timedelta
from typing import Callable

import torch
import torch.distributed as dist

NCCL_PREFIX = "_ptype/nccl"


def node_id(local_addr: str, port: int) -> str:
    return f"{local_addr}:{int(port)}"


def alive_nodes(registry, service: str, timeout_s: float = 30.0) -> list[str]:
    """Sorted ``address:port`` of the service's nodes with a live lease; retries
    while the control plane itself is electing."""
    from ..cluster import background

    deadline = time.monotonic() + timeout_s
    while True:
        try:
            nodes = registry.Services(background()).get(service, [])
            return sorted({node_id(n.address, n.port) for n in nodes})
        except Exception:
            if time.monotonic() > deadline:
                raise
            time.sleep(0.1)


def wait_nodes(registry, service: str, world: int, timeout_s: float = 60.0) -> list[str]:
    """The first ``world`` registered nodes of ``service`` (sorted), once there are that many."""
    deadline = time.monotonic() + timeout_s
    while True:
        nodes = alive_nodes(registry, service, timeout_s)
        if len(nodes) >= world:
            return nodes[:world]
        if time.monotonic() > deadline:
            raise TimeoutError(f"only {len(nodes)} of {world} data-plane nodes of {service!r} registered")
        time.sleep(0.05)


def form_group(store, local_addr: str, me: str, service: str, epoch: int, proposal: list[str], backend: str,
               device_for_rank: Callable[[int], torch.device | None] = lambda r: None, timeout_s: float = 10.0,
               rdv_timeout_s: float = 60.0):
    """Rendezvous ``proposal`` through ``store`` (a ``cluster.KVStore``) and
    initialise the default (gloo) process group.  Returns ``(members, tcp_store)``;
    keep ``tcp_store`` alive for the group's lifetime (the master serves it)."""
    if backend != "gloo":
        raise ValueError("form_group forms gloo groups (CPU runtimes); GPU data planes are NativeGroups")
    from ..cluster import SortAscend, SortByCreateRevision, WithPrefix, WithSort, background
    from .elastic import Excluded

    prefix = f"{NCCL_PREFIX}/{service}/{epoch}/"
    mine = None
    if proposal and proposal[0] == me:  # candidate rendezvous master
        mine = dist.TCPStore(local_addr, 0, len(proposal), True, timeout=timedelta(seconds=rdv_timeout_s),
                             wait_for_workers=False)
        store.Put(background(), prefix + me, json.dumps({"addr": local_addr, "port": mine.port, "members": proposal}))
    deadline = time.monotonic() + rdv_timeout_s
    rec = None
    while rec is None:
        try:
            vals = store.Get(background(), prefix, WithPrefix(), WithSort(SortByCreateRevision, SortAscend))
            rec = json.loads(vals[0]) if vals else None
        except Exception:  # ErrNoKey until a candidate publishes
            rec = None
        if rec is None:
            if time.monotonic() > deadline:
                raise TimeoutError(f"no data-plane epoch {epoch} of {service!r} published")
            time.sleep(0.05)
    members = rec["members"]
    if me not in members:
        raise Excluded(f"{me} was left out of data-plane epoch {epoch}: {members}")
    rank = members.index(me)
    leader = rank == 0 and mine is not None and rec["port"] == mine.port
    tcp = mine if leader else dist.TCPStore(rec["addr"], int(rec["port"]), len(members), False,
                                            timeout=timedelta(seconds=rdv_timeout_s))
    dist.init_process_group(backend, store=dist.PrefixStore(f"ptype/{service}/epoch{epoch}", tcp), rank=rank,
                            world_size=len(members), timeout=timedelta(seconds=timeout_s))
    return members, tcp

"""GPU-side service replication (SURVEY 2.4 "service replication", the DP analog).

The reference serves one service from several nodes and a client spreads its
calls over them (cluster/rpc.go): it SELECTS nodes -- all of them when
``MaxConnections`` is 0 or at least the node count, otherwise
``nodes[FNV-1a32(localAddr + itoa(i)) % n]`` for i = 0, 1, ... (duplicates
allowed, rpc.go:246-270) -- and takes the selected ones ROUND ROBIN, the first
call going to index 1 (rpc.go:176-183).  Two ``prime_worker`` replicas are the
example (example/optimus/worker/prime_worker*.yaml).

On the GPU data plane a replicated stateless service is hosted by several
ranks, each holding the same logical actors ``[0, n)`` in its mailboxes
``[0, n)``: global actor id ``a * W + rank`` of the group's strided id space, so
the route kernels' affine directory resolves it with no extra lookup.  A
replica publishes a lease-attached record ``_ptype/actors/<service>/<node>``
with ``"replica": true`` and its net/rpc address; a client's ``ReplicaRouter``
follows those records (``RegistryMirror`` without a table: records only),
selects with the host balancer's own ``ConnectionBalancer.select_nodes`` (the
same FNV picks, in registry key order) and routes each message on the device
(``replica_route`` kernel, csrc/hip/batch.hip): message i of a Send whose
counter starts at ``seq`` goes to ``sel[(seq + 1 + i) % len(sel)]``, then the
counter advances by the batch size -- exactly the ranks a per-call round robin
would have picked, one kernel per Send.  A replica whose lease lapses leaves
the selection at the router's next refresh (every Send applies the mirror), so
its calls move to the survivors.
"""
from __future__ import annotations

import torch

from ..ops import hip


def select_ranks(local_addr: str, records: list[dict], max_connections: int) -> list[int]:
    """The ranks a client at ``local_addr`` selects among replica ``records``
    (sorted by registry key), by the host balancer's rule."""
    from .._core import ConnectionBalancer, Node

    nodes = [Node(str(r["address"]), int(r["port"])) for r in records]
    by_node = {(str(r["address"]), int(r["port"])): int(r["rank"]) for r in records}
    sel = ConnectionBalancer.select_nodes(local_addr, nodes, int(max_connections))
    return [by_node[(n.address, n.port)] for n in sel]


class ReplicaRouter:
    """Per-client replica selection + device routing for one replicated service.

    ``kv`` + ``service``: follow the service's replica records (watch + re-list,
    mirror.py); or ``records=[...]`` for a fixed set (``set_records`` replaces
    it).  ``world`` is the group's (original) world: the id space's stride."""

    def __init__(self, service: str, world: int, local_addr: str, max_connections: int = 3, kv=None,
                 records: list[dict] | None = None, watch: bool = True):
        self.service, self.world, self.local_addr = service, int(world), local_addr
        self.max_connections = int(max_connections)
        self.seq = 0  # calls routed so far (the balancer's round-robin counter)
        self.mirror = None
        self._records: list[dict] = []
        self.sel: list[int] = []
        self.n_logical = 0
        self._sel_dev = {}
        if kv is not None:
            from ..mirror import RegistryMirror

            self.mirror = RegistryMirror(None, kv, service, watch=watch)
        if records is not None:
            self.set_records(records)
        else:
            self.refresh()

    def set_records(self, records: list[dict]) -> None:
        recs = sorted((r for r in records if r.get("replica")), key=lambda r: str(r.get("node", "")))
        self._records = recs
        self.sel = select_ranks(self.local_addr, recs, self.max_connections) if recs else []
        self.n_logical = min((int(r["count"]) for r in recs), default=0)
        self._sel_dev = {}

    def refresh(self) -> None:
        """Apply the mirror (replica joins / lease lapses) and re-select."""
        if self.mirror is None:
            return
        if self.mirror.apply() or not self._records:
            self.set_records([sh["record"] for _, sh in sorted(self.mirror.shards.items())])

    def route(self, actor: torch.Tensor) -> torch.Tensor:
        """Global actor ids (int32) for logical ids ``actor``, replica chosen per
        message; advances the round-robin counter by the batch size."""
        self.refresh()
        if not self.sel:
            raise RuntimeError(f"no replicas of {self.service!r} registered")
        M = actor.numel()
        out = torch.empty(M, dtype=torch.int32, device=actor.device)
        if actor.device.type == "cuda":
            a = actor.to(torch.int32).contiguous()
            hip().replica_route(a.data_ptr(), out.data_ptr(), M, self.sel, self.seq, self.world, self.n_logical,
                                torch.cuda.current_stream(actor.device).cuda_stream)
        else:  # the host data plane: the same rule with torch ops
            key = str(actor.device)
            if key not in self._sel_dev:
                self._sel_dev[key] = torch.tensor(self.sel, dtype=torch.int64, device=actor.device)
            sel = self._sel_dev[key]
            j = (self.seq + 1 + torch.arange(M, dtype=torch.int64, device=actor.device)) % len(self.sel)
            a = actor.to(torch.int64)
            out = torch.where((a >= 0) & (a < self.n_logical), a * self.world + sel[j], -1).to(torch.int32)
        self.seq += M
        return out

    def close(self) -> None:
        if self.mirror is not None:
            self.mirror.close()

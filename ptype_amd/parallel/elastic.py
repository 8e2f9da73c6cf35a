"""Elastic data plane: rank-failure detection and recovery for the exchange.

SURVEY 5.3.  The reference detects failed service nodes by **lease expiry**
(2 s TTL + KeepAlive, cluster/registry.go:59-83) observed through a watch, and
clients re-balance onto the survivors (cluster/rpc.go:197-244).  The data plane
is a communicator over the service's GPUs (RCCL over xGMI, or IpcComm between
the processes of one GPU) and a collective with a dead peer fails or stalls.
RCCL is not fault tolerant, so a generation is never repaired in place -- it is
aborted and a new one formed:

1. ``send`` fails (a peer's failure, or the Send watchdog's deadline) -> the
   survivor aborts the generation,
2. waits until the control plane's lease-based membership (the service's
   registry nodes) drops the dead node (bounded by ``grace_s``),
3. re-rendezvouses through the replicated KV store: the record with the lowest
   create revision under ``_ptype/nccl/<svc>/<gen>/`` wins, so candidates with
   different views still converge on one member list,
4. re-homes the dead rank's actors by a deterministic ring adoption (the next
   surviving original rank adopts them into extra mailbox blocks; actors of live
   ranks never move and keep their state), rebuilds the GPU registry mirror, and
5. the caller's batch is re-sent: delivery is at-least-once, as with the
   reference client's retries (rpc.go:107-116).

On a GPU every step of that is compiled: ``_core.DataPlane``
(csrc/core/dataplane.cpp: watchdog thread, abort, settle, form, ring adoption,
buddies, replica moves), driven through ``NativeGroup``.  A CPU runtime (gloo,
for tests and GPU-less hosts) runs the same steps with the Python helpers below
(``settle_membership``, ``ring_placement``, ``buddy``, ``lost_blocks``) over a
torch gloo group re-formed by ``bootstrap.form_group``.  ``ElasticDataPlane`` is
the standalone form (its own table and exchange, no registry mirror).

Actor state survives a rank loss through **buddy replicas** kept in HBM:
``replicate()`` (collective; also every ``replicate_every`` sends) ships every
block a node hosts to its *buddy* -- the next surviving node after it in the
original ring, by construction the node ``ring_placement`` makes adopt those
blocks -- with one send / receive pair per neighbour.  An adopted block resumes
from its replica; a block with no replica (two neighbours lost at once) restarts
from zero.  The control plane itself survives the loss of a minority of members
(Raft quorum).
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

from ..ops import batch as B
from ..ops.table import RegistryTable, actor_keys
from .exchange import ActorExchange



class RankFailure(RuntimeError):
    """A collective of the current data-plane generation failed."""


class Excluded(RuntimeError):
    """This node is not a member of the newest generation."""


# What a collective raises when a PEER failed, as opposed to a local error (CUDA
# OOM, a launch failure, a stalled look-back), which must propagate unchanged
# instead of aborting the whole group: gloo's transport errors carry
# their source path, RCCL's entry points are named in the engines' messages
# (csrc/hip/engine.hpp, exchange_sorted.hip, ipc_comm.hpp), and torch raises its
# Dist* errors for both backends.
_PEER_FAILURE_MARKS = ("gloo/transport", "Connection closed by peer", "Connection reset by peer", "Broken pipe",
                       "ncclAllToAll failed", "ncclAllReduce failed", "ncclSend failed", "ncclRecv failed",
                       "ncclGroupEnd failed", "ncclGroupStart failed", "ncclRemoteError", "ncclSystemError",
                       "IpcComm: peer", "FakeComm: a rank did not reach")


def is_rank_failure(e: BaseException) -> bool:
    """Whether ``e`` (raised by a data-plane collective) means a peer rank failed."""
    import torch.distributed as dist

    if isinstance(e, RankFailure):
        return True
    for name in ("DistBackendError", "DistNetworkError", "DistStoreError"):
        t = getattr(dist, name, None)
        if t is not None and isinstance(e, t):
            return True
    msg = str(e)
    return any(m in msg for m in _PEER_FAILURE_MARKS)


def ring_placement(nodes0: list[str], members: list[str]) -> dict[str, list[int]]:
    """Original rank -> owner: every surviving node owns its own original rank
    first, then adopts each dead original rank whose next surviving successor
    (in original ring order) it is.  Returns ``{node: [original ranks]}``."""
    alive = set(members)
    own = {n: ([r] if n in alive else []) for r, n in enumerate(nodes0)}
    W0 = len(nodes0)
    for r, n in enumerate(nodes0):
        if n in alive:
            continue
        for k in range(1, W0):
            succ = nodes0[(r + k) % W0]
            if succ in alive:
                own[succ].append(r)
                break
    return {n: rs for n, rs in own.items() if n in alive}


def buddy(nodes0: list[str], members: list[str], node: str) -> str:
    """The next surviving node after ``node`` in original ring order: the one
    ``ring_placement`` hands ``node``'s blocks to if ``node`` dies."""
    alive = set(members)
    i = nodes0.index(node)
    for k in range(1, len(nodes0)):
        n = nodes0[(i + k) % len(nodes0)]
        if n in alive:
            return n
    return node


def abort_group() -> None:
    """Tear down a gloo group of a failed generation (CPU runtimes).  Never raises."""
    if dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:
            pass


def settle_membership(alive, members: list[str], me: str, grace_s: float) -> list[str]:
    """The next generation's proposal after a collective failed: wait (at most
    ``grace_s``) until the lease-based membership ``alive()`` has dropped
    somebody of ``members`` (the dead node's 2 s registry lease lapsing), then
    keep the survivors in their old order (so ranks stay dense and ordered)."""
    old = set(members)
    deadline = time.monotonic() + grace_s
    live = alive()
    while set(live) >= old and time.monotonic() < deadline:  # nobody's lease has expired yet
        time.sleep(0.1)
        live = alive()
    proposal = [n for n in members if n in set(live)]
    if me not in proposal:
        proposal = sorted(set(proposal) | {me})
    return proposal


def lost_blocks(nodes0: list[str], before: list[str], after: list[str]) -> list[int]:
    """Original ranks whose host in generation ``before`` is not in ``after``."""
    own = ring_placement(nodes0, before)
    gone = set(before) - set(after)
    return sorted(r for n in gone for r in own.get(n, []))


class ElasticDataPlane:
    """Batched ``Send`` over a self-healing data plane.

    ``cluster`` is a joined ``ptype_amd.cluster.Cluster`` (its node is
    registered under ``service``); ``world`` the number of data-plane ranks
    expected at start; ``per_rank`` actors hosted per original rank (actor ``a``
    belongs to original rank ``a % world``, mailbox ``a // world``).  On a GPU
    the generations are the compiled DataPlane's (``NativeGroup``: ``backend``
    "native", RCCL); on the CPU a torch gloo group.
    """

    def __init__(self, cluster, service: str, world: int, per_rank: int, device=None, backend: str | None = None,
                 max_batch: int = 1 << 20, chunks: int = 1, timeout_s: float = 10.0, grace_s: float = 8.0,
                 rendezvous_timeout_s: float = 60.0, replicate_every: int = 0):
        self.cluster = cluster
        self.service = service
        self.world0 = int(world)
        self.per_rank = int(per_rank)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.backend = backend or ("native" if self.device.type == "cuda" else "gloo")
        if self.backend not in ("native", "gloo"):
            raise ValueError("backend: 'native' (the compiled DataPlane, GPU) or 'gloo' (CPU)")
        self.max_batch = int(max_batch)
        self.chunks = int(chunks)
        self.timeout_s = float(timeout_s)
        self.grace_s = float(grace_s)
        self.rdv_timeout_s = float(rendezvous_timeout_s)
        self.me = f"{cluster.local_addr}:{cluster.cfg.port}"
        self.gen = -1
        self.nodes0: list[str] = []
        self.members: list[str] = []
        self.blocks: list[int] = []  # original ranks whose actors this node hosts, in mailbox-block order
        self.state: torch.Tensor | None = None
        self.table: RegistryTable | None = None
        self.exchange: ActorExchange | None = None
        self.group = None  # NativeGroup (backend "native")
        self._tcp_store = None
        self.recoveries = 0
        self.replicate_every = int(replicate_every)
        self.replicas: dict[int, torch.Tensor] = {}  # original rank -> its block as of the last replicate()
        self.restored: list[int] = []  # blocks the last re-formation resumed from a replica
        self._sends = 0

    # ------------------------------------------------------------------ membership
    def alive(self, timeout_s: float = 30.0) -> list[str]:
        """Nodes of the service whose registry lease is alive (control plane).
        Retries while the control plane itself is re-electing."""
        from .bootstrap import alive_nodes

        return alive_nodes(self.cluster.Registry, self.service, timeout_s)

    def start(self) -> None:
        """Wait for ``world`` registered nodes and form generation 0."""
        if self.backend == "native":
            from .native_group import NativeGroup

            self.group = NativeGroup.join(self.cluster._c, self.service, self.me, lambda r: self.device, self.world0,
                                          timeout_s=self.rdv_timeout_s)
            self.nodes0 = list(self.group.dp.nodes0)
            self.gen, self.members = self.group.gen, self.group.members
            self._rebuild(dict(self.group.dp.placement(self.members)))
            return
        deadline = time.monotonic() + self.rdv_timeout_s
        while True:
            nodes = self.alive()
            if len(nodes) >= self.world0:
                break
            if time.monotonic() > deadline:
                raise TimeoutError(f"only {len(nodes)} of {self.world0} data-plane nodes registered")
            time.sleep(0.05)
        self.nodes0 = nodes[: self.world0]
        if self.me not in self.nodes0:
            raise Excluded(f"{self.me} is not among the first {self.world0} nodes of {self.service}")
        self._form(0, self.nodes0)

    def _form(self, gen: int, proposal: list[str]) -> None:
        from .bootstrap import form_group

        members, store = form_group(self.cluster.Store, self.cluster.local_addr, self.me, self.service, gen,
                                    proposal, self.backend, lambda r: None,
                                    timeout_s=self.timeout_s, rdv_timeout_s=self.rdv_timeout_s)
        self._tcp_store = store  # the master keeps the store alive for the group's lifetime
        self.gen, self.members = gen, members
        self._rebuild(ring_placement(self.nodes0, self.members))

    # ------------------------------------------------------------------ placement
    def _rebuild(self, own: dict) -> None:
        W0, P = self.world0, self.per_rank
        new_blocks = list(own[self.me])
        state = torch.zeros(P * len(new_blocks), dtype=torch.int64, device=self.device)
        self.restored = []
        if self.state is not None:  # actors that stay here keep their state
            for j, r in enumerate(new_blocks):
                if r in self.blocks:
                    i = self.blocks.index(r)
                    state[j * P:(j + 1) * P] = self.state[i * P:(i + 1) * P]
                elif r in self.replicas:  # adopted: resume from the buddy replica
                    state[j * P:(j + 1) * P] = self.replicas[r]
                    self.restored.append(r)
        self.blocks, self.state = new_blocks, state
        self.replicas = {}  # the ring changed: replicas are re-taken by the next replicate()
        table = RegistryTable(2 * W0 * P, device=self.device)
        k = torch.arange(P, dtype=torch.int64)
        for node, rs in own.items():
            rank = self.members.index(node)
            for j, r in enumerate(rs):
                ids = r + W0 * k
                table.upsert(actor_keys(ids), torch.full((P,), rank, dtype=torch.int32), (j * P + k).to(torch.int32))
        table.enable_directory(W0 * P, affine_world=W0)
        self.table = table
        self.exchange = ActorExchange(table, self.max_batch, chunks=self.chunks, state=self.state, group=self.group)

    @property
    def total_actors(self) -> int:
        return self.world0 * self.per_rank

    # ------------------------------------------------------------------ data plane
    def send(self, batch: B.MsgBatch):
        """One ``send_all`` in the current generation; a collective failure
        surfaces as ``RankFailure`` (the group is then unusable)."""
        try:
            return self.exchange.send_all(batch)
        except Exception as e:  # gloo/RCCL errors come as RuntimeError / DistBackendError
            raise RankFailure(f"generation {self.gen}: {e}") from e

    def send_resilient(self, batch: B.MsgBatch, max_recoveries: int = 3):
        """``send`` + recover-and-resend on rank failure (at-least-once);
        replicates state every ``replicate_every`` successful sends."""
        for attempt in range(max_recoveries + 1):
            try:
                out = self.send(batch)
            except RankFailure:
                if attempt == max_recoveries:
                    raise
                self.recover()
                continue
            self._sends += 1
            if self.replicate_every and self._sends % self.replicate_every == 0:
                try:
                    self.replicate()
                except RankFailure:
                    # the batch WAS delivered: recover the group, never re-send it
                    # (non-commutative methods would run twice -- ADVICE r2)
                    self.recover()
            return out

    def replicate(self) -> None:
        """Collective over the current generation: every node sends the blocks
        it hosts to its buddy and keeps the blocks of the node whose buddy it is,
        as resident device tensors.  Point-to-point only (two neighbours)."""
        P = self.per_rank
        try:
            if self.group is not None:
                dp = self.group.dp
                src_blocks = list(dp.replica_blocks())
                recv = torch.empty(max(1, P * len(src_blocks)), dtype=torch.int64, device=self.device)
                torch.cuda.current_stream(self.device).synchronize()
                got = list(dp.replicate(self.state.data_ptr(), self.state.numel() * 8, recv.data_ptr(),
                                        P * len(src_blocks) * 8))
                self.replicas = {r: recv[j * P:(j + 1) * P] for j, r in enumerate(got)}
                return
            own = ring_placement(self.nodes0, self.members)
            dst = buddy(self.nodes0, self.members, self.me)
            if dst == self.me:  # alone: nothing can adopt these blocks
                return
            src = next(n for n in self.members if buddy(self.nodes0, self.members, n) == self.me)
            recv = torch.empty(P * len(own[src]), dtype=torch.int64, device=self.device)
            ops = [dist.P2POp(dist.isend, self.state, self.members.index(dst)),
                   dist.P2POp(dist.irecv, recv, self.members.index(src))]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            self.replicas = {r: recv[j * P:(j + 1) * P] for j, r in enumerate(own[src])}
        except Exception as e:
            raise RankFailure(f"generation {self.gen}: replicate: {e}") from e

    def recover(self) -> None:
        """Abort the failed generation, wait for the lease-driven membership to
        settle, form the next generation from the survivors, re-home actors."""
        self.exchange = None
        self.recoveries += 1
        if self.group is not None:  # compiled: abort, settle, form, ring adoption
            plan = self.group.recover(self.grace_s)
            self.gen, self.members = self.group.gen, list(plan["members"])
            self._rebuild(dict(self.group.dp.placement(self.members)))
            return
        abort_group()
        proposal = settle_membership(self.alive, self.members, self.me, self.grace_s)
        self._form(self.gen + 1, proposal)

    def close(self) -> None:
        if self.group is not None:
            self.group.close()
            self.group = None
        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass
        self._tcp_store = None

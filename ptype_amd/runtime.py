"""Per-process GPU actor runtime: the device side of a cluster member.

One process per GPU.  A ``DeviceRuntime`` owns, on its GPU:

* the actor mailboxes' state (``int64`` per actor, random-init optional),
* the persistent dispatcher (host-visible request/reply rings) for the
  single-call latency path -- ``Call`` on a GPU actor needs no kernel launch,
* the GPU registry mirror (``ops.RegistryTable``) mapping every actor id of a
  service to (rank, mailbox), kept in step with the authoritative control-plane
  store, and
* the exchange engine (``parallel.ActorExchange``) for batched ``Send`` across
  the GPUs of the node over RCCL.

Actor placement is published in the replicated KV store, one key per rank and
service (``store/_ptype/actors/<service>/<node>`` -> ``{"rank","world","count"}``,
strided ids: actor ``a`` lives on rank ``a % world`` in mailbox ``a // world``),
attached to a lease this process keeps alive, so the Raft log carries one
entry per shard, not one per actor, while the GPU table holds every actor (1M
actors = 2M slots = 32 MB of HBM).  ``mirror.RegistryMirror`` follows those
records (watch + lease expiry) into the table; with ``gpu.world > 1`` Join
forms the data-plane group through the store first (parallel/bootstrap.py).

Rank failures.  A runtime whose group Join formed is elastic.  On
a GPU the group is the compiled DataPlane (``NativeGroup``: RCCL, or IpcComm
between the processes of one GPU) and the whole lifecycle is its: the Send
watchdog (a C++ thread) fails a generation whose Send is overdue, ``recover``
is one call -- abort, lease-driven settle, generation g + 1 through the store,
ring adoption of the lost ranks' blocks -- and ``replicate`` moves buddy
replicas; this module only applies the DataPlane's plan to its tensors (the
state blocks, the registry table, the dispatcher).  A CPU runtime (gloo)
re-forms its torch group the same way (bootstrap.form_group, elastic.py
helpers).  Either way the dead rank's actors move to their ring successor
(state from the buddy replica, else zero), the shard record is republished and
the Send is re-sent:
``send_all`` re-sends the whole batch (at-least-once, like the reference
client's retries, cluster/rpc.go:107-116); ``send(..., resend_overflow=False)``
answers the messages whose actor lived on the lost rank with
``STATUS_RANK_LOST`` and delivers the rest.  The reference's client survives a
dead node the same way: lease lapse (cluster/registry.go:51-86), watch re-list
(:119-150), balancer re-selection (cluster/rpc.go:197-244).

Reference: the reference has no device side; this realises SURVEY C9/C10/C14
under the API of cluster/cluster.go and cluster/rpc.go.
"""
from __future__ import annotations

import json
import logging
import os
import time

import torch

from .ops import batch as B
from .ops import hip
from .ops.records import STATUS_OK, STATUS_RANK_LOST
from .ops.table import RegistryTable, actor_keys
from .utils import trace

ACTORS_PREFIX = "_ptype/actors"
_log = logging.getLogger("ptype.runtime")


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


class DeviceRuntime:
    def __init__(self, device=None, actors: int = 1024, ring: int = 4096, idle_ms: float = 200.0,
                 delay_us: int = 0, max_batch: int = 1 << 20, chunks: int = 0, random_state: bool = False,
                 group=None, shm: bool = True, service: str = "", mailbox_shards: int = 256,
                 mailbox_slots: int = 0, delivery: str = "auto", comm: str = "rccl", comm_timeout_s: float = 30.0):
        if device is None:
            device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        self.device = torch.device(device)
        # a CPU runtime runs the handler table's host reference (tests, GPU-less hosts):
        # no persistent dispatcher, no HBM mailboxes, gloo collectives
        self.on_gpu = self.device.type == "cuda"
        if self.on_gpu:
            torch.cuda.set_device(self.device)
        d = _dist()
        self.group = group
        if group is not None and hasattr(group, "comm_ptr"):  # NativeGroup: the compiled DataPlane
            self.rank, self.world = group.rank, group.size
        else:
            self.rank = d.get_rank(group) if d else 0
            self.world = d.get_world_size(group) if d else 1
        self.service = service
        # services whose actors are this runtime's actors: the one it joined as, plus
        # any co-hosted through host()/serve() (one actor id space per runtime)
        self.hosted: set[str] = {service} if service else set()
        self.actors = int(actors)
        if random_state:
            g = torch.Generator(device=self.device).manual_seed(1234 + self.rank)
            self.state = torch.randint(0, 1 << 20, (self.actors,), dtype=torch.int64, device=self.device, generator=g)
        else:
            self.state = torch.zeros(self.actors, dtype=torch.int64, device=self.device)
        self.delay_us = int(delay_us)
        self.server = None
        if self.on_gpu:
            # dispatcher rings in shared memory: same-node client processes call these
            # GPU actors without a socket (shmring.hpp)
            self.server = hip().DeviceServer(self.device.index or 0, int(ring), self.state.data_ptr(), self.actors,
                                             self.delay_us, float(idle_ms), 60.0,
                                             f"ptype-{os.getpid()}-{self.device.index or 0}" if shm else "")
        self._ring, self._idle_ms = int(ring), float(idle_ms)
        self.table = RegistryTable(2 * self.actors * self.world, device=self.device)
        # dense actor ids [0, actors*world): route through the compiled directory (K5b)
        self.table.enable_directory(self.actors * self.world, affine_world=self.world)
        self.max_batch = int(max_batch)
        # 2 pipeline chunks at N > 1: the measured optimum at R = 2, 4 and 8 (profiles/r2_chunk_model)
        self.chunks = chunks or (1 if self.world == 1 else 2)
        # elasticity (set by for_cluster when Join formed the group)
        self.world0 = self.world    # the original world: actor a belongs to original rank a % world0
        self.blocks = [self.rank]   # original ranks whose actors this process hosts (mailbox-block order)
        self.membership = None      # {"me", "nodes0", "members", "gen"} of the group Join formed
        self._elastic_cfg = None
        self.replicas: dict[int, torch.Tensor] = {}  # original rank -> its block as of the last replicate()
        self.restored: list[int] = []
        self.recoveries = 0
        self.replicate_every = 0
        self._sends = 0
        self._cpu_failed = None  # a CPU runtime's failed generation (fail_generation)
        self.mailbox_shards, self.mailbox_slots = int(mailbox_shards), int(mailbox_slots)
        self.delivery = delivery or "auto"  # "mailbox": every Send through the HBM mailboxes (ActorExchange)
        # N > 1 collectives: the group's RCCL communicator, or IpcComm ("ipc": shared-memory
        # segments every rank maps, over a gloo group -- several ranks may share one GPU)
        self.comm, self.comm_timeout_s = comm or "rccl", float(comm_timeout_s)
        self._exchange = None
        self.shards: dict[str, list[dict]] = {}
        self.mirror = None  # RegistryMirror (watch-driven) once attached to a control plane
        self.shard_lease = None
        self._tcp_store = None  # rendezvous store of a group this runtime formed (kept alive)
        self._owns_group = False
        self._closed = False

    # ------------------------------------------------------------------ setup
    @classmethod
    def for_cluster(cls, core_cluster, cfg) -> "DeviceRuntime":
        """The device side of ``Join``: form the service's data plane through the
        store when ``gpu.world > 1`` (parallel/bootstrap.py), start the runtime on
        this rank's device, publish the actor shard under a lease and mirror every
        shard of the service into the registry table (mirror.py)."""
        import torch.distributed as dist

        from .cluster import KVStore, Registry

        g = cfg.gpu
        owns = False
        tcp = None
        ndev = 0 if g.cpu else torch.cuda.device_count()

        def device_for_rank(r: int):
            if g.cpu:
                return torch.device("cpu")
            if g.device >= 0:
                return torch.device("cuda", g.device)
            lr = os.environ.get("LOCAL_RANK")
            return torch.device("cuda", int(lr) if lr is not None else r % max(ndev, 1))

        members = None
        native = None
        if (g.world > 1 or g.form_group) and not (dist.is_available() and dist.is_initialized()):
            from .parallel.bootstrap import form_group, node_id, wait_nodes

            me = node_id(core_cluster.local_addr, cfg.port)
            registry = Registry(core_cluster.registry)
            store = KVStore(core_cluster.store)
            if not g.cpu:
                # the group's whole lifecycle in the control plane (csrc/core/dataplane.hpp): store
                # rendezvous, RCCL init (or IpcComm segments: gpu.comm ipc), abort, next generation
                from .parallel.exchange import ipc_cap_for
                from .parallel.native_group import NativeGroup

                world = max(g.world, 1)
                chunks = 1 if world == 1 else 2
                native = NativeGroup.join(core_cluster, cfg.service_name, me, device_for_rank, world,
                                          timeout_s=max(30.0, g.group_timeout_s), transport=g.comm,
                                          cap_bytes=ipc_cap_for(g.max_batch, chunks, world) if g.comm == "ipc" else 0)
                members = native.members
                backend = "native"
            else:
                backend = g.backend or "gloo"
                nodes = wait_nodes(registry, cfg.service_name, max(g.world, 1))
                members, tcp = form_group(store, core_cluster.local_addr, me, cfg.service_name, 0, nodes, backend,
                                          device_for_rank, timeout_s=g.group_timeout_s)
            owns = True
        d = _dist()
        rank = native.rank if native is not None else (d.get_rank() if d else 0)
        rt = cls(device_for_rank(rank), actors=g.actors, ring=g.ring, idle_ms=g.idle_ms, delay_us=g.delay_us,
                 max_batch=g.max_batch, service=cfg.service_name, mailbox_shards=g.mailbox_shards,
                 mailbox_slots=g.mailbox_slots, delivery=g.delivery, comm=g.comm,
                 comm_timeout_s=g.group_timeout_s, group=native)
        rt._tcp_store, rt._owns_group = tcp, owns
        rt._addr = (core_cluster.local_addr, int(cfg.port))
        if members is not None and g.elastic:
            rt.membership = {"me": me, "nodes0": list(members), "members": list(members), "gen": 0}
            rt._elastic_cfg = {"store": store, "registry": registry, "local_addr": core_cluster.local_addr,
                               "backend": backend, "timeout_s": g.group_timeout_s, "grace_s": g.grace_s,
                               "max_recoveries": 3}
            rt.replicate_every = int(g.replicate_every)
            if g.send_timeout_s > 0 and native is not None:  # the DataPlane's watchdog thread (C++)
                native.dp.set_watchdog(float(g.send_timeout_s))
        rt.attach(core_cluster.registry.kv, cfg.service_name, cfg.node_name, watch=g.watch)
        # Send needs every rank's routes: wait until all shards of the group are mirrored
        rt.mirror.wait_shards(rt.world)
        return rt

    def attach(self, kv, service: str, node: str, watch: bool = True) -> None:
        """Publish this rank's shard (lease-attached) and follow every shard of
        ``service`` into the registry table."""
        from .mirror import RegistryMirror, ShardLease

        self.service = service
        self.hosted.add(service)
        self.shard_lease = ShardLease(kv, service, node, self.rank, self.world, self.actors)
        self.table.clear()
        self.mirror = RegistryMirror(self.table, kv, service, watch=watch)
        self.mirror.apply()
        self._kv, self._node = kv, node

    def sync(self) -> int:
        """Apply pending registry changes (joins, leaves, lease expiries) now."""
        return self.mirror.apply() if self.mirror is not None else 0

    def publish_shard(self, store, service: str, node: str) -> None:
        """Record this rank's actor shard of `service` in the replicated store
        (without a lease; ``attach`` keeps a lease-attached record instead)."""
        from .cluster import Context

        v = json.dumps({"rank": self.rank, "world": self.world, "count": self.actors, "node": node})
        store.put(Context.background(), f"{ACTORS_PREFIX}/{service}/{node}", v)

    def sync_registry(self, store, service: str) -> int:
        """One-shot rebuild of the GPU registry mirror of `service` from the
        published shards (K5 batch upsert on the device); returns the number of actors."""
        from .cluster import Context, NoKeyError, WithPrefix

        try:
            vals = store.get(Context.background(), f"{ACTORS_PREFIX}/{service}/", WithPrefix())
        except NoKeyError:
            vals = []
        shards = [json.loads(v) for v in vals]
        self.shards[service] = shards
        self.table.clear()
        total = 0
        for s in shards:
            n, r, w = int(s["count"]), int(s["rank"]), int(s["world"])
            mbox = torch.arange(n, dtype=torch.int64, device=self.device)
            ids = r + w * mbox
            self.table.upsert(actor_keys(ids), torch.full((n,), r, dtype=torch.int32, device=self.device),
                              mbox.to(torch.int32))
            total += n
        return total

    def place_local(self, n_actors_total: int | None = None) -> None:
        """Strided placement without a control plane (single process / bench):
        every rank mirrors every rank's shard."""
        n = self.actors
        self.table.clear()
        for r in range(self.world):
            mbox = torch.arange(n, dtype=torch.int64, device=self.device)
            self.table.upsert(actor_keys(r + self.world * mbox),
                              torch.full((n,), r, dtype=torch.int32, device=self.device), mbox.to(torch.int32))

    @property
    def total_actors(self) -> int:
        return self.actors * self.world0

    @property
    def mailboxes(self) -> int:
        """Mailboxes this process hosts (``actors`` per hosted block)."""
        return self.state.numel()

    @property
    def exchange(self):
        if self._exchange is None:
            from .parallel.exchange import ActorExchange

            self._exchange = ActorExchange(self.table, self.max_batch, chunks=self.chunks, group=self.group,
                                           state=self.state, delay_us=self.delay_us, delivery=self.delivery,
                                           mailbox_shards=self.mailbox_shards, mailbox_slots=self.mailbox_slots,
                                           comm=self.comm if self.on_gpu else "rccl",
                                           comm_timeout_s=self.comm_timeout_s)
        return self._exchange

    # ------------------------------------------------------------------ data plane
    def host(self, service: str) -> None:
        """Co-host ``service`` on this runtime's actors (the reference registers
        several net/rpc services on one server; here they share the GPU actors and
        the registry mirror, and a Send names which one it addresses)."""
        self.hosted.add(service)

    def _check_service(self, service: str | None) -> None:
        if service and self.hosted and service not in self.hosted:
            raise ValueError(f"Send to {service!r}: this process's data plane hosts {sorted(self.hosted)} "
                             "(co-host more services with DeviceRuntime.host)")

    # ------------------------------------------------------------------ replicated services (parallel/replicas.py)
    def serve_replica(self, service: str, address: str | None = None, port: int | None = None) -> None:
        """Serve ``service`` as one replica of a replicated stateless service:
        its logical actors [0, actors) are this rank's mailboxes (lease-attached
        record ``_ptype/actors/<service>/<node>`` with ``"replica": true``)."""
        from .mirror import ShardLease

        if getattr(self, "_kv", None) is None:
            raise RuntimeError("serve_replica needs a control plane (Join, or attach())")
        addr, p = self._addr if getattr(self, "_addr", None) else ("", 0)
        self.host(service)
        lease = ShardLease(self._kv, service, self._node, self.blocks[0], self.world0, self.actors, replica=True,
                           address=address if address is not None else addr, port=int(port if port is not None else p))
        self._replica_leases = getattr(self, "_replica_leases", {})
        self._replica_leases[service] = lease

    def has_replicas(self, service: str) -> bool:
        """Whether ``service`` has replica records in the store."""
        from .mirror import ACTORS_PREFIX, STORE_PREFIX, _prefix_end

        kv = getattr(self, "_kv", None)
        if kv is None:
            return False
        from ._core import RangeOpts

        o = RangeOpts()
        pfx = f"{STORE_PREFIX}{ACTORS_PREFIX}/{service}/"
        o.end = _prefix_end(pfx)
        return any(json.loads(x.value).get("replica") for x in kv.get(pfx, o).kvs)

    def replica_router(self, service: str, max_connections: int = 3, local_addr: str | None = None):
        """A client's replica selection for ``service`` (follows its records)."""
        from .parallel.replicas import ReplicaRouter

        la = local_addr if local_addr is not None else (self._addr[0] if getattr(self, "_addr", None) else "")
        return ReplicaRouter(service, self.world0, la, max_connections, kv=self._kv)

    def send(self, service: str | None, batch: B.MsgBatch, resend_overflow: bool = True, router=None):
        """Batched Send: every message to its actor anywhere in the node and the
        replies back in message order.  Collective across the process group.
        Registry changes seen since the last Send are applied first.  With an
        elastic group a rank failure is recovered here (module docstring).
        ``router``: a replicated service's ReplicaRouter -- the batch's logical
        actor ids are routed to the selected replicas, round robin."""
        if router is not None:
            batch = B.MsgBatch(router.route(batch.actor), batch.a0, batch.a1, batch.a2, batch.method)
        else:
            self._check_service(service)
        self.sync()
        if self.membership is None:
            ex = self.exchange
            # more than one rank: no host wait on this Send (its overflow, if any, is
            # re-sent just before Send + 2 or at flush(): ActorExchange.send_all)
            return ex.send_all(batch, defer=self.world > 1) if resend_overflow else ex.send(batch)
        from .parallel.elastic import RankFailure, is_rank_failure

        dp = self.group.dp if self._native else None  # the compiled lifecycle (watchdog, recovery)
        lost_before: list[int] = []
        todo = None  # after a recovery without re-sends: the indices still to deliver
        for attempt in range(self._elastic_cfg["max_recoveries"] + 1):
            try:
                if self._failed():
                    raise RankFailure(self._failed())
                sub = batch if todo is None else batch.index_select(todo)
                if dp is not None:
                    dp.begin_send()  # the host part of the Send is bounded too
                try:
                    out = self.exchange.send_all(sub) if resend_overflow else self.exchange.send(sub)
                finally:
                    if dp is not None:
                        dp.end_send()
                if dp is not None and dp.watchdog_failed:  # aborted mid-Send: its replies are void
                    raise RankFailure(dp.watchdog_failed)
                ipc = self.exchange.ipc
                if ipc is not None:  # IpcComm: a peer that missed a collective is seen once the Send's waits end
                    torch.cuda.current_stream(self.device).synchronize()
                    ipc.check()
            except RuntimeError as e:
                # only a peer's failure re-forms the group; a local error (OOM, a launch
                # failure, a stalled look-back) propagates unchanged -- recovering from it
                # would abort every rank and re-run delivered, non-commutative messages
                if not is_rank_failure(e) or attempt == self._elastic_cfg["max_recoveries"]:
                    raise
                _log.warning("data-plane generation %d failed: %s", self.membership["gen"], str(e)[:300])
                trace.mark("ptype.rank_failure")
                lost_before += self.recover()
                if not resend_overflow and lost_before:
                    # messages whose actor lived on a lost rank: STATUS_RANK_LOST, not re-run
                    a = batch.actor.to(torch.int64)
                    lost = torch.zeros(a.numel(), dtype=torch.bool, device=a.device)
                    for r in lost_before:
                        lost |= (a % self.world0) == r
                    todo = torch.nonzero(~lost).flatten()
                continue
            self._sends += 1
            if dp is not None and self.on_gpu:  # the Send's device work must finish in time
                dp.arm(torch.cuda.current_stream(self.device).cuda_stream)
            if self.replicate_every and self._sends % self.replicate_every == 0:
                try:
                    self.replicate()
                except RuntimeError as e:
                    if not is_rank_failure(e):
                        raise
                    self.recover()  # the batch WAS delivered: recover, never re-send it
            if todo is None:
                return out
            val = torch.zeros(batch.M, dtype=out[0].dtype, device=out[0].device)
            st = torch.full((batch.M,), STATUS_RANK_LOST, dtype=out[1].dtype, device=out[1].device)
            val[todo] = out[0]
            st[todo] = out[1]
            return (val, st) + tuple(out[2:])
        raise AssertionError("unreachable")

    def _failed(self) -> str:
        """Why the current generation was failed ("" while fine)."""
        return self.group.dp.watchdog_failed if self._native else (self._cpu_failed or "")

    def fail_generation(self, why: str) -> None:
        """Mark the current generation failed, as the Send watchdog does: the next
        Send recovers (fault injection of the tests)."""
        if self._native:
            self.group.dp.fail_generation(why)
        else:
            self._cpu_failed = why

    def flush(self) -> None:
        """Every earlier Send's replies final (deferred re-sends run now).  Collective."""
        if getattr(self, "_exchange", None) is not None:
            self._exchange.flush()

    # ------------------------------------------------------------------ rank failures
    def replicate(self) -> None:
        """Collective over the current generation: every rank ships the blocks it
        hosts to its buddy (the node that would adopt them) and keeps the blocks it
        is buddy of, resident in HBM.  Point-to-point only.  On a GPU the DataPlane
        picks the buddies and moves the bytes (csrc/core/dataplane.cpp replicate)."""
        import torch.distributed as dist

        from .parallel.elastic import buddy, ring_placement

        m = self.membership
        if m is None:
            return
        P = self.actors
        if self._native:
            dp = self.group.dp
            src_blocks = list(dp.replica_blocks())
            recv = torch.empty(max(1, P * len(src_blocks)), dtype=torch.int64, device=self.device)
            torch.cuda.current_stream(self.device).synchronize()  # the state's producers are done
            st = self.state.contiguous()
            got = list(dp.replicate(st.data_ptr(), st.numel() * 8, recv.data_ptr(), P * len(src_blocks) * 8))
            self.replicas = {r: recv[j * P:(j + 1) * P] for j, r in enumerate(got)}
            return
        own = ring_placement(m["nodes0"], m["members"])
        dst = buddy(m["nodes0"], m["members"], m["me"])
        if dst == m["me"]:
            return
        src = next(n for n in m["members"] if buddy(m["nodes0"], m["members"], n) == m["me"])
        # a gloo group (CPU runtimes) moves host tensors
        recv = torch.empty(P * len(own[src]), dtype=torch.int64, device=self.device)
        ops = [dist.P2POp(dist.isend, self.state, m["members"].index(dst)),
               dist.P2POp(dist.irecv, recv, m["members"].index(src))]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        self.replicas = {r: recv[j * P:(j + 1) * P] for j, r in enumerate(own[src])}

    def recover(self) -> list[int]:
        """Abort the failed generation, let the lease-based membership settle,
        form the next generation through the store and re-home the lost ranks'
        actors.  Returns the original ranks that were lost."""
        from .parallel.bootstrap import alive_nodes, form_group
        from .parallel.elastic import Excluded, lost_blocks, ring_placement, settle_membership

        m, c = self.membership, self._elastic_cfg
        if m is None:
            raise RuntimeError("recover(): this runtime's group was not formed by Join")
        self._abort_generation()
        if self._exchange is not None and self._exchange.pending():
            # (elastic Sends never defer; a deferred Send of the failed generation keeps
            # STATUS_OVERFLOW on its pending messages -- say so instead of dropping it silently)
            _log.warning("recover: %d deferred Send(s) of generation %d left unresolved (STATUS_OVERFLOW)",
                         self._exchange.drop_pending(), m["gen"])
        self._exchange = None
        if self._native:
            # the compiled lifecycle: abort, lease-driven settle, the first current record in
            # the store wins, the next generation's communicator, ring adoption
            dp = self.group.dp
            try:
                plan = self.group.recover(float(c["grace_s"]))
            except RuntimeError as e:
                if "excluded" in str(e):
                    raise Excluded(str(e)) from e
                raise
            dp.reset_watchdog()
            lost = list(plan["lost"])
            m["members"], m["gen"] = list(plan["members"]), m["gen"] + 1
            self.rank, self.world = self.group.rank, self.group.size
            own = {n: list(rs) for n, rs in dict(dp.placement(m["members"])).items()}
            self._rehome(own, list(plan["blocks"]), list(plan["kept_from"]), list(plan["from_replica"]))
        else:
            proposal = settle_membership(lambda: alive_nodes(c["registry"], self.service), m["members"], m["me"],
                                         c["grace_s"])
            members, tcp = form_group(c["store"], c["local_addr"], m["me"], self.service, m["gen"] + 1, proposal,
                                      c["backend"], lambda r: None, timeout_s=c["timeout_s"])
            self._tcp_store = tcp
            self._cpu_failed = None
            lost = lost_blocks(m["nodes0"], m["members"], members)
            m["members"], m["gen"] = list(members), m["gen"] + 1
            self.rank, self.world = members.index(m["me"]), len(members)
            own = ring_placement(m["nodes0"], m["members"])
            nb = own[m["me"]]
            kept = [self.blocks.index(r) if r in self.blocks else -1 for r in nb]
            self._rehome(own, nb, kept, [k < 0 and r in self.replicas for r, k in zip(nb, kept)])
        self.recoveries += 1
        _log.warning("data-plane generation %d formed: world %d, lost original ranks %s, hosting %s", m["gen"],
                     self.world, lost, self.blocks)
        trace.mark("ptype.regenerated")
        return lost

    @property
    def _native(self) -> bool:
        """Whether the group is the compiled DataPlane (parallel/native_group.py)."""
        return self.group is not None and hasattr(self.group, "comm_ptr")

    def _abort_generation(self) -> None:
        """Abort the current data-plane generation (never raises)."""
        if self._native:
            try:
                self.group.abort()
            except Exception:
                pass
        else:
            from .parallel.elastic import abort_group

            abort_group()

    def _rehome(self, own: dict, new_blocks: list, kept_from: list, from_replica: list) -> None:
        """Apply a placement: keep the state of blocks that stay, adopt lost blocks
        from their replicas (else zero), rebuild the registry table and the
        dispatcher, republish this rank's record.  ``own``: node -> original ranks."""
        m = self.membership
        P, W0 = self.actors, self.world0
        state = torch.zeros(P * len(new_blocks), dtype=torch.int64, device=self.device)
        self.restored = []
        for j, (r, k, rep) in enumerate(zip(new_blocks, kept_from, from_replica)):
            if k >= 0:
                state[j * P:(j + 1) * P] = self.state[k * P:(k + 1) * P]
            elif rep and r in self.replicas:
                state[j * P:(j + 1) * P] = self.replicas[r]
                self.restored.append(r)
        self.blocks, self.state, self.replicas = list(new_blocks), state, {}
        self.table.clear()
        k = torch.arange(P, dtype=torch.int64)
        for node, rs in own.items():
            rank = m["members"].index(node)
            for j, r in enumerate(rs):
                self.table.upsert(actor_keys(r + W0 * k), torch.full((P,), rank, dtype=torch.int32),
                                  (j * P + k).to(torch.int32))
        self.table.enable_directory(W0 * P, affine_world=W0)
        self._ltable = None
        if self.server is not None:  # the dispatcher serves the new state tensor
            name = self.server.shm_name
            self.server.close()
            self.server = hip().DeviceServer(self.device.index or 0, self._ring, self.state.data_ptr(),
                                             self.mailboxes, self.delay_us, self._idle_ms, 60.0, name)
        for _, b in getattr(self, "_bridges", []):  # the net/rpc server keeps their handles: retarget in place
            b.retarget(self.table.table.data_ptr(), self.table.cap, self.state.data_ptr(), self.state.numel())
        if self.mirror is not None:
            self.mirror.set_generation(m["gen"])
        if self.shard_lease is not None:
            self.shard_lease.update(rank=self.rank, world=W0, count=P, gen=m["gen"], blocks=list(new_blocks))

    def tell(self, batch: B.MsgBatch, outbox_capacity: int | None = None):
        """Fire-and-forget delivery that lets GPU handlers send on: ``batch`` is
        delivered, and whatever the handlers emit (actor-to-actor ``Forward``
        tells) is routed epoch after epoch until every outbox of the group is
        empty.  Collective.  Returns ``(epochs, messages delivered here)``."""
        from .ops.outbox import DeviceOutbox

        cap = int(outbox_capacity or self.max_batch)
        if getattr(self, "_outbox", None) is None or self._outbox.cap < cap:
            self._outbox = DeviceOutbox(cap, device=self.device)
        return self.exchange.pump(self._outbox, initial=batch)

    def call(self, method: int, actor: int, a0: int = 0, a1: int = 0, a2: int = 0, timeout: float = 30.0):
        """Single synchronous call to a local actor.  Through the persistent
        dispatcher (no kernel launch) -- except ordered methods, which must queue
        behind the actor's other messages: those go through its HBM mailbox."""
        from .ops.records import method_ordered

        if not self.on_gpu or method_ordered(method):
            b = B.MsgBatch(torch.tensor([actor], dtype=torch.int32, device=self.device),
                           torch.tensor([a0], dtype=torch.int64, device=self.device),
                           torch.tensor([a1], dtype=torch.int64, device=self.device),
                           torch.tensor([a2], dtype=torch.int64, device=self.device), int(method))
            if self.on_gpu:
                mb = self.exchange._mailboxes()
                v, st = mb.send(b, self._local_table(), self.state, rank_self=0, delay_us=self.delay_us, ordered=True)
                return int(v.item()), int(st.item())
            v, st = B._handler_ref(torch.tensor([int(method)]), torch.tensor([actor]), b.a0, b.a1, b.a2, self.state)
            return int(v[0]), int(st[0])
        with trace.range("ptype.call"):
            v, st, _ = self.server.call(int(method), int(actor), int(a0), int(a1), int(a2), float(timeout))
        return v, st

    def _local_table(self):
        """Identity table of this rank's mailboxes (a local call names the mailbox)."""
        if getattr(self, "_ltable", None) is None:
            t = RegistryTable(2 * self.actors, device=self.device)
            ids = torch.arange(self.actors, dtype=torch.int64)
            t.upsert(actor_keys(ids), torch.zeros(self.actors, dtype=torch.int32), ids.to(torch.int32))
            t.enable_directory(self.actors)
            self._ltable = t
        return self._ltable

    def serve(self, server, service: str, methods: dict, batch: bool = False) -> None:
        """Expose GPU handlers over net/rpc: ``methods`` maps a Go method name to
        ``(method_id, [arg field names])`` -- e.g. ``{"Multiply": (1, ["A", "B"])}``.
        ``batch``: also serve each method in batches through the GPU gob bridge
        (K4: a connection's pipelined requests decoded on the GPU into mailbox
        columns, ``gob_bridge``)."""
        self.host(service)
        if batch and self.world0 > 1:
            # the bridge routes with mailbox = actor id on this GPU: right only when
            # this rank hosts every actor
            raise ValueError("serve(batch=True): the GPU gob bridge serves single-rank runtimes only")
        for name, (mid, fields) in methods.items():
            server.RegisterDevice(f"{service}.{name}", self.server, mid, fields)
            if batch:
                server.RegisterDeviceBatch(f"{service}.{name}", self.gob_bridge(mid).handle(), fields)

    def gob_bridge(self, method_id: int, actor: int = 0):
        """The GPU gob bridge of ``method_id`` (csrc/hip/gob_bridge.hpp): batches
        of gob argument messages decoded on this GPU and sent through mailboxes of
        their own (separate rings: the bridge runs on its own stream), answering
        actor ``actor`` (or the request's actor field).  Kept alive by the runtime."""
        from .ops.mailbox import Mailboxes

        if not self.on_gpu:
            raise RuntimeError("gob_bridge needs a GPU runtime (use _core.host_batch_multiply() on the host)")
        self._bridges = getattr(self, "_bridges", [])
        mb = Mailboxes(self.device, shards=64, slots=1 << 12)
        # ordered after the runtime's stream both ways: a bridge batch and a Send never
        # update actor state concurrently
        b = hip().GobBridge(self.device.index or 0, mb._m, int(method_id), int(actor), self.table.table.data_ptr(),
                            self.table.cap, self.state.data_ptr(), self.state.numel(), self.delay_us,
                            torch.cuda.current_stream(self.device).cuda_stream)
        self._bridges.append((mb, b))
        return b

    # ------------------------------------------------------------------ snapshots (C14)
    def snapshot_to_host(self) -> dict:
        """Actor state + packed registry mirror in pinned host DRAM, on a side
        stream (the routing stream keeps running): the state by one DMA copy, the
        mirror by K7 writing straight into its pinned buffers.  The pinned
        buffers are allocated once and reused; the returned tensors are views
        valid until the next snapshot."""
        side = torch.cuda.Stream(self.device) if self.on_gpu else None
        if self.on_gpu:
            side.wait_stream(torch.cuda.current_stream(self.device))
            if getattr(self, "_snap_state", None) is None or self._snap_state.numel() != self.state.numel():
                self._snap_state = torch.empty(self.state.shape, dtype=self.state.dtype, pin_memory=True)
            with torch.cuda.stream(side):
                self._snap_state.copy_(self.state, non_blocking=True)
            h_state = self._snap_state
        else:
            h_state = self.state.clone()
        ent, exp = self.table.snapshot_to_host(side)
        return {"state": h_state, "table": ent, "expiry": exp,
                "meta": torch.tensor([self.rank, self.world, self.actors], dtype=torch.int64)}

    def save(self, path: str) -> dict:
        from safetensors.torch import save_file

        t0 = time.perf_counter()
        snap = self.snapshot_to_host()
        nbytes = sum(v.numel() * v.element_size() for v in snap.values())
        save_file({k: v.contiguous() for k, v in snap.items()}, path)
        return {"bytes": nbytes, "seconds": time.perf_counter() - t0}

    def restore(self, path: str) -> None:
        from safetensors.torch import load_file

        snap = load_file(path)
        if int(snap["meta"][2]) != self.actors:
            raise ValueError("snapshot actor count does not match this runtime")
        self.restore_from(snap)

    def restore_from(self, snap: dict) -> None:
        """Actor state and registry mirror from a snapshot dict (``snapshot_to_host``
        output): one host->device copy each, the mirror re-inserted by one packed
        upsert kernel."""
        pin = self.on_gpu and not snap["state"].is_pinned()
        st = snap["state"].pin_memory() if pin else snap["state"]
        self.state.copy_(st, non_blocking=self.on_gpu)
        self.table.clear()
        if snap["table"].numel():
            ent, exp = snap["table"], snap["expiry"]
            if self.on_gpu and not ent.is_pinned():
                ent, exp = ent.pin_memory(), exp.pin_memory()
            self.table.load_packed(ent, exp)

    # ------------------------------------------------------------------ stats / teardown
    def stats(self) -> dict:
        from dataclasses import asdict

        from .utils.trace import hist_percentile

        out = {"rank": self.rank, "world": self.world, "actors": self.actors, "device": str(self.device)}
        if self.server is not None:
            h = self.server.rtt_histogram()
            out["dispatcher"] = {"processed": self.server.processed, "launches": self.server.launches,
                                 "exits_idle": self.server.exits_idle, "exits_lifetime": self.server.exits_lifetime,
                                 "running": self.server.running, "calls": int(sum(h)),
                                 "rtt_p50_ns_le": hist_percentile(h, 50), "rtt_p99_ns_le": hist_percentile(h, 99),
                                 "rtt_log2ns_hist": h}
        out["registry"] = {"live": self.table.live, "tombstones": self.table.tombstones,
                           "generation": self.table.generation, "capacity": self.table.cap,
                           "directory_ids": self.table.dir_n}
        out["shards"] = ({k: v["record"] for k, v in self.mirror.shards.items()} if self.mirror is not None
                         else self.shards)
        if self.mirror is not None:
            out["mirror"] = {"applies": self.mirror.applies, "actors": self.mirror.actors}
        if self._exchange is not None:
            out["exchange"] = asdict(self._exchange.stats())
        return out

    def close(self) -> None:
        if self._closed:
            return
        self._closed = True
        if self._exchange is not None and self._exchange.pending():
            # deferred re-sends (world > 1) resolve before the group goes away (collective:
            # every rank closes); a failure here is reported, the teardown goes on
            try:
                self._exchange.flush()
            except Exception as e:  # noqa: BLE001
                _log.warning("close: deferred re-sends not resolved: %s", str(e)[:300])
        for lease in getattr(self, "_replica_leases", {}).values():
            lease.close()
        if self.mirror is not None:
            self.mirror.close()
        if self.shard_lease is not None:
            self.shard_lease.close()
        if self.server is not None:
            self.server.close()
        if self._owns_group and self._native:
            self.group.close()  # abort: never waits on a member that may be gone
        elif self._owns_group:
            import torch.distributed as dist

            if dist.is_initialized():
                try:
                    dist.destroy_process_group()
                except Exception:
                    pass
            self._tcp_store = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def verify_ok(status: torch.Tensor) -> bool:
    return bool((status == STATUS_OK).all())

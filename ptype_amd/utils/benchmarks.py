"""Secondary measurements of ``bench.py`` (BASELINE.json configs 4 and 5, and the
public API path), each a dict that bench.py puts under ``secondaries``.

* ``registry_1m``: the 1M-actor GPU registry mirror (K5 inserts / updates /
  lookups, K5b directory build, K6 sweep scan) and its snapshot into pinned host
  DRAM (K7) and restore -- BASELINE config 5 (reference: the etcd keyspace of
  cluster/registry.go:51-86, here mirrored in HBM).
* ``optimus_fanout``: the optimus coordinator for many targets per step -- one
  Send of every target's 10-wide ranges (coordinator.go:67-73) through the
  node's data plane (the sorted exchange at N > 1) and the device gather
  (coordinator.go:91-98, csrc/hip/optimus.hip) -- BASELINE config 4, with the
  reference's 250 ms per-candidate delay set to 0 as BASELINE.md prescribes.
* ``api_send``: ``Join -> NewClient -> Client.Send`` eager, the whole public
  API path (control-plane member, registry mirror apply, send_all) around the
  same mailbox Send as the headline.

Every timing brackets its steps with device synchronisation (and, with a
process group, barriers) and verifies the replies outside the timed loop."""
from __future__ import annotations

import os
import socket
import tempfile
import time

import torch


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def static_ports(rank: int, world: int, offset: int) -> tuple[int, int, int, str]:
    """(peer port, client port, service port, initial-cluster string) of rank
    ``rank`` in a static ``world``-member cluster on 127.0.0.1 that every rank
    derives alike from MASTER_PORT (+ ``offset``: one cluster per purpose)."""
    base = int(os.environ.get("MASTER_PORT", "29500")) + offset
    if base + 3 * world >= 65536:
        base = 20000 + base % 20000
    pp, pc, port = base + 2 * rank, base + 2 * rank + 1, base + 2 * world + rank
    initial = ",".join(f"b{r}=http://127.0.0.1:{base + 2 * r}" for r in range(world))
    return pp, pc, port, initial


def bench_group(device, rank: int, world: int, comm: str = "rccl", cap_bytes: int = 0, service: str = "bench",
                offset: int = 211, timeout_s: float = 120.0):
    """The bench's data plane at N > 1 the way ``Join`` forms it: a control-plane
    member per rank (a static cluster on 127.0.0.1), and the compiled DataPlane's
    communicator over the service's registered nodes -- RCCL, or IpcComm for a
    one-GPU rehearsal -- with no torch process group (reference
    cluster/cluster.go:28-84).  Returns ``(cluster, NativeGroup)``."""
    from .. import cluster as C
    from ..parallel.native_group import NativeGroup

    os.environ.setdefault("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    pp, pc, port, initial = static_ports(rank, world, offset)
    cfg = C.Config()
    cfg.service_name, cfg.node_name, cfg.port = service, f"r{rank}", port
    cfg.member = C.member_config(name=f"b{rank}", dir=tempfile.mkdtemp(prefix="ptype_benchdp_"),
                                 lpurls=[f"http://127.0.0.1:{pp}"], apurls=[f"http://127.0.0.1:{pp}"],
                                 lcurls=[f"http://127.0.0.1:{pc}"], acurls=[f"http://127.0.0.1:{pc}"],
                                 initial_cluster=initial, unsafe_no_fsync=True)
    c = C.Join(C.background(), cfg, runtime=False)
    try:
        g = NativeGroup.join(c._c, service, f"{c._c.local_addr}:{port}", lambda r: device, world,
                             timeout_s=timeout_s, transport=comm, cap_bytes=cap_bytes)
    except Exception:
        c.Close()
        raise
    if g.rank != rank:  # (ranks follow the sorted node ids: the same order as RANK)
        raise RuntimeError(f"data-plane rank {g.rank} != launcher rank {rank}")
    return c, g


def kv_barrier(cluster, key: str, world: int, timeout_s: float = 120.0) -> None:
    """A host-side barrier through the replicated store: no collective kernel on
    any GPU while it waits (peers' dispatchers may need to launch meanwhile)."""
    from .. import cluster as C

    rank = int(os.environ.get("RANK", "0"))
    st = cluster.Store
    st.Put(C.background(), f"_barrier/{key}/{rank}", "1")
    t_end = time.monotonic() + timeout_s
    while time.monotonic() < t_end:
        try:
            if len(st.Get(C.background(), f"_barrier/{key}/", C.WithPrefix(), C.WithKeysOnly())) >= world:
                return
        except Exception:  # (ErrNoKey before the first put lands)
            pass
        time.sleep(0.002)
    raise TimeoutError(f"kv_barrier {key}: not every rank arrived")


def timed(step, steps: int, warmup: int, device, barrier=None) -> float:
    """Seconds for ``steps`` calls of ``step`` after ``warmup`` untimed ones."""
    for _ in range(warmup):
        step()
    _sync(device)
    if barrier:
        barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    _sync(device)
    if barrier:
        barrier()
    return time.perf_counter() - t0


# ---------------------------------------------------------------------------- config 5
def registry_1m(device, n: int = 1 << 20, reps: int = 5) -> dict:
    from ..ops.table import RegistryTable, actor_keys

    out = {"config": "1M-actor GPU registry mirror + snapshot to pinned host DRAM", "actors": n}
    keys = actor_keys(torch.arange(n, dtype=torch.int64)).to(device)
    ranks = (torch.arange(n, device=device) % 8).to(torch.int32)
    mbox = (torch.arange(n, device=device) // 8).to(torch.int32)
    exp = torch.full((n,), 1 << 40, dtype=torch.int64, device=device)
    ins = []
    t = None
    for _ in range(reps):  # inserts into an empty table (allocation outside the timed region)
        t = RegistryTable(2 * n, device=device)
        _sync(device)
        t0 = time.perf_counter()
        t.upsert(keys, ranks, mbox, exp)
        _sync(device)
        ins.append(time.perf_counter() - t0)
    out["insert_ops_per_s"] = n / min(ins)
    out["update_ops_per_s"] = n / (timed(lambda: t.upsert(keys, ranks, mbox, exp), reps, 1, device) / reps)
    q = keys[torch.randperm(n, device=device)]
    out["lookup_ops_per_s"] = n / (timed(lambda: t.lookup(q), reps, 1, device) / reps)
    t.enable_directory(n)

    def build_dir():
        t._dir_dirty = True
        t.directory()

    out["directory_build_ms"] = timed(build_dir, reps, 1, device) / reps * 1e3
    out["sweep_scan_ms"] = timed(lambda: t.sweep(1), reps, 1, device) / reps * 1e3
    side = torch.cuda.Stream(device)
    h_ent, h_exp = t.snapshot_to_host(side)  # pinned buffers allocated once, reused
    els = []
    for _ in range(reps):
        _sync(device)
        t0 = time.perf_counter()
        h_ent, h_exp = t.snapshot_to_host(side)
        els.append(time.perf_counter() - t0)
    nbytes = h_ent.numel() * 8 + h_exp.numel() * 8
    out["snapshot_bytes"] = nbytes
    out["snapshot_to_pinned_ms"] = min(els) * 1e3
    out["snapshot_gb_per_s"] = nbytes / min(els) / 1e9
    rest = []
    for _ in range(3):
        t2 = RegistryTable(2 * n, device=device)
        _sync(device)
        t0 = time.perf_counter()
        t2.load_packed(h_ent, h_exp)
        _sync(device)
        rest.append(time.perf_counter() - t0)
        if t2.live != n:
            raise RuntimeError(f"registry restore: {t2.live} of {n} entries")
    out["restore_ms"] = min(rest) * 1e3
    if not all(torch.equal(a, b) for a, b in zip(t.lookup(q), t2.lookup(q))):
        raise RuntimeError("registry restore: lookups differ from the snapshotted table")
    return out


# ---------------------------------------------------------------------------- config 4
def optimus_max_batch(world: int, targets: int = 1024, base: int = 80_001, sets: int = 3) -> int:
    """The largest batch ``optimus_fanout`` sends on any rank (its exchange's
    geometry -- e.g. the IpcComm region size a bench group must be formed with):
    target t is ceil(t / 10) ranges, and the last rank's last set has the largest."""
    tg = torch.arange(targets, dtype=torch.int64) * 2 + base + ((world - 1) + (sets - 1) * world) * 2 * targets
    return int(((tg + 9) // 10).sum())


def optimus_fanout(table, n_actors: int, device, steps: int, warmup: int, rank: int = 0, world: int = 1,
                   targets: int = 1024, base: int = 80_001, chunks: int = 1, comm: str = "rccl", barrier=None,
                   max_over_ranks=None, sets: int = 3, group=None) -> dict:
    """``targets`` odd numbers per rank and set (distinct per rank and set), every
    one split into 10-wide ranges and answered by the Prime.Check actors of the
    whole node; the answers are checked against trial division on a sample.
    Steps cycle over ``sets`` distinct batches (~230 MB each at the defaults):
    more than the 256 MB MALL, so no step reads a batch the cache still holds."""
    from ..models.optimus import FanOut
    from ..ops.records import STATUS_OK
    from ..parallel.exchange import ActorExchange

    fs = []
    for j in range(sets):
        tg = torch.arange(targets, dtype=torch.int64) * 2 + base + (rank + j * world) * 2 * targets
        fs.append((tg, FanOut(tg, n_actors, device)))
    Mx = max(f.M for _, f in fs)
    ex = ActorExchange(table, Mx, chunks=chunks, delivery="mailbox", mailbox_ordered=False, comm=comm, group=group)
    val = torch.empty(Mx, dtype=torch.int64, device=device)
    st = torch.empty(Mx, dtype=torch.int32, device=device)
    k = [0]

    def step():
        f = fs[k[0] % sets][1]
        k[0] += 1
        ex.send(f.batch, val[:f.M], st[:f.M])
        f.gather(val[:f.M], st[:f.M])

    for tg, f in fs:  # every set once, checked
        step()
        _sync(device)
        if not bool((f.status == STATUS_OK).all()):
            raise RuntimeError("optimus fan-out: a range failed")
        for j in range(0, targets, max(1, targets // 32)):
            t = int(tg[j])
            want = next((d for d in range(2, int(t ** 0.5) + 2) if t % d == 0 and d < t), t)
            if int(f.answer[j]) != want:
                raise RuntimeError(f"optimus fan-out: target {t} answered {int(f.answer[j])}, expected {want}")
    k0 = k[0] + warmup  # the first timed step's set
    el = timed(step, steps, warmup, device, barrier)
    if max_over_ranks is not None:
        el = max_over_ranks(el)
    M = sum(fs[(k0 + i) % sets][1].M for i in range(steps))  # the timed steps' ranges
    bbytes = sum(f.M * 28 for _, f in fs)  # actor 4 + three int64 columns per range
    return {"config": "example/optimus fan-out + device gather (delay 0)", "targets_per_gpu_per_step": targets,
            "ranges_per_gpu_per_step": M // max(steps, 1), "value": M * world / el,
            "unit": "ranges/s (Prime.Check messages, whole node)", "targets_per_s": targets * world * steps / el,
            "ms_per_step": el / steps * 1e3, "delivery": "mailbox" + (" (sorted exchange)" if world > 1 else ""),
            "gather": "device (first non-target reply per target, early exit)",
            "distinct_batches": sets, "batch_bytes_total": bbytes}


# ---------------------------------------------------------------------------- public API
def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def api_send(device, sizes, actors: int, steps: int, warmup: int, rank: int = 0, world: int = 1,
             comm: str = "rccl", barrier=None, max_over_ranks=None) -> dict:
    """Join (a control-plane member, GPU runtime, lease-attached shard, registry
    mirror) -> NewClient -> Client.Send of pre-generated batches, eager, through
    the HBM mailboxes (gpu.delivery: mailbox).  With ``world`` > 1: one member
    per rank in a static cluster on 127.0.0.1 (ports from MASTER_PORT), whose
    Join forms the service's data plane (the compiled DataPlane: RCCL, or IpcComm
    with ``comm="ipc"``), and every rank Sends its own batches to actors all over
    the node (the sorted exchange, deferred re-sends: no host wait per Send); the
    timed loop ends with ``Client.Flush``, and the slowest rank's time counts."""
    from .. import cluster as C
    from ..ops import batch as B
    from ..ops.records import METHOD_CALC_MULTIPLY, STATUS_OK

    os.environ.setdefault("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    cfg = C.Config()
    if world > 1:  # every rank derives the same static cluster from the rendezvous port
        pp, pc, port, initial = static_ports(rank, world, 1237)
    else:
        pp, pc, port = _port(), _port(), _port()
        initial = f"b0=http://127.0.0.1:{pp}"
    cfg.service_name, cfg.node_name, cfg.port = "calculator", f"bench{rank}", port
    cfg.member = C.member_config(name=f"b{rank}", dir=tempfile.mkdtemp(prefix="ptype_bench_"),
                                 lpurls=[f"http://127.0.0.1:{pp}"], apurls=[f"http://127.0.0.1:{pp}"],
                                 lcurls=[f"http://127.0.0.1:{pc}"], acurls=[f"http://127.0.0.1:{pc}"],
                                 initial_cluster=initial, unsafe_no_fsync=True)
    cfg.has_gpu = True
    g = cfg.gpu
    g.device, g.actors, g.max_batch, g.delivery = device.index or 0, actors, max(sizes), "mailbox"
    g.world, g.comm = world, comm
    g.cpu = device.type == "cpu"  # (the CPU twin of the path, for tests)
    t0 = time.perf_counter()
    srv = C.Serve(cfg.port, _Host(), host="127.0.0.1")  # the node's net/rpc server (what NewClient dials)
    c = C.Join(C.background(), cfg)
    out = {"path": "Join -> NewClient -> Client.Send (eager, mailbox delivery, pre-generated batches)",
           "join_s": time.perf_counter() - t0, "ranks": world}
    try:
        client = c.NewClient("calculator", C.ConnConfig(retries=0, allow_local=False))
        n_ids = c.runtime.total_actors  # every rank's actors
        for M in sizes:
            # at least 3 distinct batches, together more than the 256 MB MALL (20 B per message)
            nb = max(3, -(-300_000_000 // (20 * M)))
            batches = [B.gen_requests(M, n_ids, METHOD_CALC_MULTIPLY, seed=11 + k + 1000 * rank, device=device)
                       for k in range(nb)]
            res = {}
            k = [0]

            def step():
                b = batches[k[0] % nb]
                k[0] += 1
                th = time.perf_counter()
                res["out"] = client.Send(b)
                res["host"] = res.get("host", 0.0) + time.perf_counter() - th
                res["b"] = b

            for _ in range(warmup):  # (first Sends of a size grow workspaces: not in the host figure)
                step()
            client.Flush()
            _sync(device)
            if barrier:
                barrier()
            res["host"] = 0.0
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            client.Flush()  # the last Sends' deferred re-sends (none in a steady state) are timed too
            _sync(device)
            if barrier:
                barrier()
            el = time.perf_counter() - t0
            if max_over_ranks is not None:
                el = max_over_ranks(el)
            host_us = res["host"] / steps * 1e6
            v, s = res["out"]
            if not (bool((s == STATUS_OK).all()) and torch.equal(v, res["b"].a0 * res["b"].a1)):
                raise RuntimeError("api_send: verification failed")
            out[f"{M}"] = {"msgs_per_step": M, "value": M * world * steps / el, "ms_per_step": el / steps * 1e3,
                           "host_us_per_send": host_us, "distinct_batches": nb, "batch_bytes_total": nb * 20 * M}
            del batches
        client.Close()
    finally:
        c.Close()
        srv.Close()
    return out


class _Host:
    """A host-side net/rpc receiver for the node's address (the balancer dials it)."""

    def Ping(self, x):
        return x

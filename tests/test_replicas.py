"""GPU data-plane service replication (parallel/replicas.py), on CPU.

* The router's per-message replica choice equals the reference client's: the
  selected nodes (all in mesh mode / when few enough, else FNV-1a32(localAddr +
  i) % n picks, cluster/rpc.go:246-270) taken round robin from index 1
  (rpc.go:176-183) -- checked against an independent FNV-1a here.
* Four gloo ranks, Prime served by replicas on ranks 1 and 3: every rank's
  CounterAdd calls land on the replicas exactly as each rank's own round robin
  picks them; Prime.Check answers are right; after one replica is lost every
  call goes to the other.
* The router follows the store: a replica whose lease lapses leaves the
  selection.
"""
import os
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port


def fnv1a32(s: str) -> int:
    h = 0x811C9DC5
    for b in s.encode():
        h = ((h ^ b) * 0x01000193) & 0xFFFFFFFF
    return h


def expected_sel(local_addr, ranks, max_conn):
    if max_conn == 0 or len(ranks) <= max_conn:
        return list(ranks)
    return [ranks[fnv1a32(local_addr + str(i)) % len(ranks)] for i in range(max_conn)]


def _records(ranks, W=4, count=16):
    return [{"rank": r, "world": W, "count": count, "node": f"p{r}", "replica": True, "address": "10.0.0.%d" % r,
             "port": 7000 + r} for r in ranks]


@pytest.mark.parametrize("max_conn", [0, 1, 2, 3])
def test_router_picks_like_the_balancer(max_conn):
    from ptype_amd.parallel.replicas import ReplicaRouter

    ranks = [0, 2, 3]
    r = ReplicaRouter("Prime", 4, "192.168.1.17", max_conn, records=_records(ranks))
    sel = expected_sel("192.168.1.17", ranks, max_conn)
    assert r.sel == sel
    seq = 0
    for M in (5, 11, 1, 64):  # several Sends: the counter carries over
        a = torch.randint(0, 16, (M,), dtype=torch.int32)
        out = r.route(a).to(torch.int64)
        want = torch.tensor([sel[(seq + 1 + i) % len(sel)] for i in range(M)])
        assert torch.equal(out % 4, want) and torch.equal(out // 4, a.to(torch.int64))
        seq += M
    # logical ids past the replicas' actors: no actor
    assert r.route(torch.tensor([16, -1], dtype=torch.int32)).tolist() == [-1, -1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ptype_amd.ops import batch as B
        from ptype_amd.ops.records import METHOD_COUNTER_ADD, METHOD_PRIME_CHECK, STATUS_NO_ACTOR, STATUS_OK
        from ptype_amd.ops.table import RegistryTable, actor_keys
        from ptype_amd.parallel.exchange import ActorExchange
        from ptype_amd.parallel.replicas import ReplicaRouter

        P = 16
        n = P * world
        table = RegistryTable(4 * n, device="cpu")
        ids = torch.arange(n)
        table.upsert(actor_keys(ids), (ids % world).to(torch.int32), (ids // world).to(torch.int32))
        table.enable_directory(n, affine_world=world)
        state = torch.zeros(P, dtype=torch.int64)
        ex = ActorExchange(table, 4096, chunks=1, state=state)
        router = ReplicaRouter("Prime", world, f"10.1.0.{rank}", 3, records=_records([1, 3], world, P))
        M = 100 + 7 * rank
        a = (torch.arange(M) % P).to(torch.int32)
        req = B.MsgBatch(router.route(a), torch.ones(M, dtype=torch.int64), None, None, METHOD_COUNTER_ADD)
        _, st = ex.send(req)
        ok1 = bool((st == STATUS_OK).all())
        # Prime.Check through the replicas: smallest divisor in [2, t) else t
        t = torch.tensor([97, 91, 2 * 31, 7 * 13 * 3], dtype=torch.int64)
        lo = torch.full_like(t, 2)
        req = B.MsgBatch(router.route(torch.arange(4, dtype=torch.int32)), lo, t, t, METHOD_PRIME_CHECK)
        val, st = ex.send(req)
        ok_prime = bool((st == STATUS_OK).all()) and val.tolist() == [97, 7, 2, 3]
        dist.barrier()
        counts1 = state.clone()
        # replica 1 lost (its record gone): the next Send goes to rank 3 only
        router.set_records(_records([3], world, P))
        req = B.MsgBatch(router.route(a), torch.ones(M, dtype=torch.int64), None, None, METHOD_COUNTER_ADD)
        _, st = ex.send(req)
        ok2 = bool((st == STATUS_OK).all())
        _, st = ex.send(B.MsgBatch(router.route(torch.tensor([P], dtype=torch.int32)), torch.ones(1, dtype=torch.int64),
                                   None, None, METHOD_COUNTER_ADD))
        ok_miss = st.tolist() == [STATUS_NO_ACTOR]
        dist.barrier()
        q.put((rank, ok1, ok_prime, ok2, ok_miss, counts1.tolist(), (state - counts1).tolist()))
    except Exception as e:
        import traceback

        q.put((rank, "error", repr(e), traceback.format_exc()[-1500:]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_replicated_service_over_four_ranks():
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in procs]
    res = sorted(q.get(timeout=90) for _ in range(world))
    [p.join(30) for p in procs]
    errs = [r for r in res if r[1] == "error"]
    assert not errs, errs
    P = 16
    # expected: each sender rank's round robin over [1, 3] (both selected: 2 <= MaxConnections)
    want1 = {1: torch.zeros(P, dtype=torch.int64), 3: torch.zeros(P, dtype=torch.int64)}
    want2 = {1: torch.zeros(P, dtype=torch.int64), 3: torch.zeros(P, dtype=torch.int64)}
    for r in range(world):
        M = 100 + 7 * r
        sel = [1, 3]
        for i in range(M):
            want1[sel[(1 + i) % 2]][i % P] += 1
        for i in range(M):  # one replica left: all of them
            want2[3][i % P] += 1
    for rank, ok1, ok_prime, ok2, ok_miss, c1, c2 in res:
        assert ok1 and ok_prime and ok2 and ok_miss, (rank, ok1, ok_prime, ok2, ok_miss)
        if rank in (1, 3):
            assert c1 == want1[rank].tolist(), (rank, c1)
            assert c2 == want2[rank].tolist(), (rank, c2)
        else:
            assert sum(c1) == 0 and sum(c2) == 0


def test_router_follows_replica_leases(tmp_path, ports, monkeypatch):
    monkeypatch.setenv("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    from ptype_amd import cluster as C
    from ptype_amd.mirror import ShardLease
    from ptype_amd.parallel.replicas import ReplicaRouter

    pp, pc = ports(), ports()
    cfg = C.Config()
    cfg.service_name, cfg.node_name, cfg.port = "svc", "n0", ports()
    cfg.member = C.member_config(name="e0", dir=str(tmp_path / "m0"), lpurls=[f"http://127.0.0.1:{pp}"],
                                 apurls=[f"http://127.0.0.1:{pp}"], lcurls=[f"http://127.0.0.1:{pc}"],
                                 acurls=[f"http://127.0.0.1:{pc}"], initial_cluster=f"e0=http://127.0.0.1:{pp}",
                                 heartbeat_ms=20, election_ms=200, unsafe_no_fsync=True)
    c = C.Join(C.background(), cfg, runtime=False)
    try:
        kv = c._c.registry.kv
        a = ShardLease(kv, "Prime", "pa", 0, 2, 8, replica=True, address="10.0.0.1", port=1)
        b = ShardLease(kv, "Prime", "pb", 1, 2, 8, replica=True, address="10.0.0.2", port=2)
        r = ReplicaRouter("Prime", 2, "10.9.9.9", 3, kv=kv)
        deadline = time.time() + 5
        while len(r.sel) < 2 and time.time() < deadline:
            time.sleep(0.05)
            r.refresh()
        assert sorted(r.sel) == [0, 1]
        assert (r.route(torch.zeros(4, dtype=torch.int32)) % 2).tolist() == [1, 0, 1, 0]
        b.stop_keepalive()  # a crash: the lease lapses
        t0 = time.time()
        while r.sel != [0] and time.time() - t0 < 8:
            time.sleep(0.1)
            r.refresh()
        assert r.sel == [0], r.sel
        assert (r.route(torch.zeros(3, dtype=torch.int32)) % 2).tolist() == [0, 0, 0]
        r.close()
        a.close()
    finally:
        c.Close()

"""Join brings up the data plane; the registry mirror follows the store.

* Three processes, each ``Join`` with a ``gpu:`` section (``cpu: true``, gloo,
  ``world: 3``) and nothing else: Join rendezvouses through the replicated store
  (parallel/bootstrap.py), every rank publishes its lease-attached actor shard
  and mirrors the others (mirror.py), and ``NewClient(svc).Send`` moves a batch
  to actors on every rank -- no torchrun, no init_process_group by the caller.
  Reference: one call joins a node (cluster/cluster.go:28-84).
* One process, two control-plane members: a node that publishes its shard
  after this runtime joined becomes routable without a manual sync, and a node
  whose lease lapses leaves the mirror within TTL + the re-list period
  (cluster/registry.go:59-83, :119-150; cluster/rpc.go:197-244).
"""
import os
import time

import pytest
import torch
import torch.multiprocessing as mp

from conftest import free_port


def _member(C, i, pp, pc, ic, tmp):
    return C.member_config(name=f"e{i}", dir=os.path.join(tmp, f"m{i}"), lpurls=[f"http://127.0.0.1:{pp[i]}"],
                           apurls=[f"http://127.0.0.1:{pp[i]}"], lcurls=[f"http://127.0.0.1:{pc[i]}"],
                           acurls=[f"http://127.0.0.1:{pc[i]}"], initial_cluster=ic, heartbeat_ms=20,
                           election_ms=200, unsafe_no_fsync=True)


class Host:
    """A host-side receiver so NewClient's balancer has a net/rpc server to dial."""

    def Ping(self, x):
        return x


def _worker(i, pp, pc, sp, tmp, q):
    os.environ["PTYPE_ADVERTISE_ADDR"] = "127.0.0.1"
    from ptype_amd import cluster as C
    from ptype_amd.ops.batch import MsgBatch
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD, STATUS_OK

    c = None
    try:
        ic = ",".join(f"e{j}=http://127.0.0.1:{pp[j]}" for j in range(3))
        cfg = C.Config()
        cfg.service_name, cfg.node_name, cfg.port = "calc", f"n{i}", sp[i]
        cfg.member = _member(C, i, pp, pc, ic, tmp)
        cfg.has_gpu = True
        cfg.gpu.cpu, cfg.gpu.world, cfg.gpu.actors, cfg.gpu.max_batch = True, 3, 32, 4096
        srv = C.Serve(sp[i], Host(), host="127.0.0.1")
        c = C.Join(C.background(), cfg)  # forms the gloo group through the store
        rt = c.runtime
        client = c.NewClient("calc", C.ConnConfig(retries=0, allow_local=False))
        n = rt.total_actors
        ids = torch.arange(n, dtype=torch.int32)
        a = ids.to(torch.int64) + 100 * i
        val, st = client.Send(MsgBatch(ids, a, torch.full((n,), 3, dtype=torch.int64), None, METHOD_CALC_MULTIPLY))
        ok_mul = bool((st == STATUS_OK).all()) and torch.equal(val, a * 3)
        # every rank adds 1 to every actor: each actor, wherever it lives, counts 3
        _, st = client.Send(MsgBatch(ids, torch.ones(n, dtype=torch.int64), None, None, METHOD_COUNTER_ADD))
        ok_add = bool((st == STATUS_OK).all())
        import torch.distributed as dist

        dist.barrier()
        q.put((i, rt.rank, rt.world, ok_mul, ok_add, bool((rt.state == 3).all()), len(rt.mirror.shards),
               client.Call("Host.Ping", "x")))
        dist.barrier()
        client.Close()
        srv.Close()
        c.Close()
    except Exception as e:
        import traceback

        q.put(("error", i, repr(e), traceback.format_exc()[-2000:]))
        if c is not None:
            c.Close()


@pytest.mark.timeout(180)
def test_join_forms_data_plane_and_send(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pp, pc, sp = ([free_port() for _ in range(3)] for _ in range(3))
    procs = [ctx.Process(target=_worker, args=(i, pp, pc, sp, str(tmp_path), q)) for i in range(3)]
    [p.start() for p in procs]
    res = [q.get(timeout=150) for _ in range(3)]
    [p.join(30) for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    errors = [r for r in res if r[0] == "error"]
    assert not errors, "\n".join("\n".join(map(str, r)) for r in errors)
    assert sorted(r[1] for r in res) == [0, 1, 2]  # ranks assigned by the rendezvous
    for i, rank, world, ok_mul, ok_add, counted, shards, ping in res:
        assert world == 3 and ok_mul and ok_add and counted and shards == 3 and ping == "x", res


def _survivor(i, pp, pc, sp, tmp, crash, q):
    """Join (world 3, elastic) -> NewClient -> Send; node ``crash`` dies without any
    cleanup after the first round; the survivors keep calling client.Send."""
    os.environ["PTYPE_ADVERTISE_ADDR"] = "127.0.0.1"
    from ptype_amd import cluster as C
    from ptype_amd.ops.batch import MsgBatch
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD, STATUS_OK, STATUS_RANK_LOST

    c = None
    try:
        ic = ",".join(f"e{j}=http://127.0.0.1:{pp[j]}" for j in range(3))
        cfg = C.Config()
        cfg.service_name, cfg.node_name, cfg.port = "calc", f"n{i}", sp[i]
        cfg.member = _member(C, i, pp, pc, ic, tmp)
        cfg.has_gpu = True
        cfg.gpu.cpu, cfg.gpu.world, cfg.gpu.actors, cfg.gpu.max_batch = True, 3, 32, 4096
        cfg.gpu.group_timeout_s, cfg.gpu.grace_s = 5.0, 10.0
        srv = C.Serve(sp[i], Host(), host="127.0.0.1")
        c = C.Join(C.background(), cfg)
        rt = c.runtime
        client = c.NewClient("calc", C.ConnConfig(retries=0, allow_local=False))
        n = rt.total_actors
        ids = torch.arange(n, dtype=torch.int32)
        add = MsgBatch(ids, torch.ones(n, dtype=torch.int64), None, None, METHOD_COUNTER_ADD)
        _, st = client.Send(add)
        ok1 = bool((st == STATUS_OK).all())
        rt.replicate()  # every block has a copy on its buddy (the node that adopts it)
        me = rt.membership["me"]
        dead = rt.membership["nodes0"][crash]
        if me == dead:
            os._exit(0)  # crash: no group teardown, no lease revoke, its Raft member gone
        # the survivors' next Send fails inside the collective and recovers underneath;
        # without re-sends, the messages of the lost rank's actors say so explicitly
        a = ids.to(torch.int64) + 100 * i
        mul = MsgBatch(ids, a, torch.full((n,), 7, dtype=torch.int64), None, METHOD_CALC_MULTIPLY)
        val, st = client.Send(mul, resend_overflow=False)
        lost = (ids % 3) == crash
        ok_lost = bool((st[lost] == STATUS_RANK_LOST).all()) and bool((st[~lost] == STATUS_OK).all()) \
            and torch.equal(val[~lost], a[~lost] * 7)
        val, st = client.Send(mul)  # re-sent: the adopter answers now
        ok2 = ok_lost and bool((st == STATUS_OK).all()) and torch.equal(val, a * 7)
        _, st = client.Send(add)
        ok3 = bool((st == STATUS_OK).all())
        import torch.distributed as dist

        dist.barrier()
        P = rt.actors
        own = sorted(int(x) for x in rt.state[:P].unique().tolist())
        adopted = sorted(int(x) for x in rt.state[P:].unique().tolist())
        q.put((me, dead, ok1, ok2, ok3, own, adopted, rt.restored, rt.world, rt.recoveries, rt.blocks,
               rt.membership["gen"], len(rt.mirror.shards)))
        dist.barrier()
        client.Close()
        srv.Close()
        c.Close()
    except Exception as e:
        import traceback

        q.put(("error", i, repr(e), traceback.format_exc()[-2500:]))
        if c is not None:
            c.Close()


@pytest.mark.timeout(240)
def test_join_send_survives_a_dead_rank(tmp_path):
    """a rank dies mid-run; the survivors' ``client.Send`` (Join ->
    NewClient -> Send, no elastic object in the test) recovers underneath:
    abort, lease-driven membership, generation 1 through the store, the dead
    rank's actors re-homed on its ring successor from the buddy replica."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pp, pc, sp = ([free_port() for _ in range(3)] for _ in range(3))
    crash = 1
    procs = [ctx.Process(target=_survivor, args=(i, pp, pc, sp, str(tmp_path), crash, q)) for i in range(3)]
    [p.start() for p in procs]
    res = [q.get(timeout=200) for _ in range(2)]
    [p.join(30) for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    errors = [r for r in res if r[0] == "error"]
    assert not errors, "\n".join("\n".join(map(str, r)) for r in errors)
    for me, dead, ok1, ok2, ok3, own, adopted, restored, world, recov, blocks, gen, shards in res:
        assert ok1 and ok2 and ok3, (me, ok1, ok2, ok3)
        assert world == 2 and recov == 1 and gen == 1, (world, recov, gen)
        assert own == [5], own  # 3 adds before the crash (one per rank), 2 after (two survivors)
        if len(blocks) > 1:  # the adopter: the dead rank's actors resumed from the replica (3) + 2
            assert blocks[1] == crash and restored == [crash] and adopted == [5], (blocks, restored, adopted)
    assert sorted(len(r[10]) for r in res) == [1, 2]  # exactly one survivor adopted the dead rank


def test_mirror_follows_joins_and_lease_expiry(tmp_path, ports, monkeypatch):
    monkeypatch.setenv("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    from ptype_amd import cluster as C
    from ptype_amd.mirror import ShardLease
    from ptype_amd.ops.table import actor_keys

    pp, pc = [ports(), ports()], [ports(), ports()]
    ic = ",".join(f"e{j}=http://127.0.0.1:{pp[j]}" for j in range(2))
    cfgs = []
    for i in range(2):
        cfg = C.Config()
        cfg.service_name, cfg.node_name, cfg.port = "calc", f"n{i}", ports()
        cfg.member = _member(C, i, pp, pc, ic, str(tmp_path))
        cfgs.append(cfg)
    import threading

    joined = [None, None]

    def join(i, rt):
        joined[i] = C.Join(C.background(), cfgs[i], runtime=rt)

    cfgs[0].has_gpu = True
    cfgs[0].gpu.cpu, cfgs[0].gpu.actors = True, 16
    ts = [threading.Thread(target=join, args=(i, i == 0)) for i in range(2)]  # static 2-member cluster
    [t.start() for t in ts]
    [t.join(30) for t in ts]
    a, b = joined
    try:
        rt = a.runtime
        # this node's shard publishes rank 0 of a 2-rank layout: ids 0, 2, 4, ...
        rt.shard_lease.close()
        rt.mirror.apply()
        mine = ShardLease(b.registry.kv, "calc", "n0", 0, 2, 16)
        rt.mirror.wait_shards(1, 10)
        rank, _ = rt.table.lookup(actor_keys(torch.tensor([4, 5])))
        assert rank.tolist() == [0, -1]  # odd ids: nobody yet
        # a node that joins later: its shard (rank 1, ids 1, 3, 5, ...) becomes routable at the next apply
        other = ShardLease(b.registry.kv, "calc", "n1", 1, 2, 16)
        deadline = time.time() + 5
        while time.time() < deadline:
            rt.sync()
            if rt.table.lookup(actor_keys(torch.tensor([5])))[0].tolist() == [1]:
                break
            time.sleep(0.05)
        rank, mbox = rt.table.lookup(actor_keys(torch.tensor([4, 5, 31])))
        assert rank.tolist() == [0, 1, 1] and mbox.tolist() == [2, 2, 15]
        # its lease lapses (no revoke: a crash) -> gone within TTL + re-list period
        other.stop_keepalive()
        t0 = time.time()
        while time.time() - t0 < 8:
            rt.sync()
            if rt.table.lookup(actor_keys(torch.tensor([5])))[0].tolist() == [-1]:
                break
            time.sleep(0.1)
        gone = time.time() - t0
        assert rt.table.lookup(actor_keys(torch.tensor([4, 5])))[0].tolist() == [0, -1]
        assert gone < 2 + 3 + 1, gone  # TTL 2 s + debounce (reference: 3 s) + slack
        assert len(rt.mirror.shards) == 1
        mine.close()
    finally:
        a.Close()
        b.Close()


def test_mirror_k6_sweeps_shards_not_seen(tmp_path, ports, monkeypatch):
    """K6 backstop: with no watch stream, a shard whose record vanished expires by
    its deadline (last seen + TTL + grace) through the table sweep."""
    monkeypatch.setenv("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    from ptype_amd import cluster as C
    from ptype_amd.mirror import RegistryMirror, ShardLease
    from ptype_amd.ops.table import RegistryTable, actor_keys

    pp, pc = ports(), ports()
    cfg = C.Config()
    cfg.service_name, cfg.node_name, cfg.port = "svc", "n0", ports()
    cfg.member = _member(C, 0, [pp], [pc], f"e0=http://127.0.0.1:{pp}", str(tmp_path))
    c = C.Join(C.background(), cfg, runtime=False)
    try:
        kv = c._c.registry.kv
        lease = ShardLease(kv, "svc", "x", 0, 1, 8)
        t = RegistryTable(64, device="cpu")
        # no watch and no re-list within the test: nothing refreshes the shard's deadline
        m = RegistryMirror(t, kv, "svc", ttl_ms=300, grace_ms=100, relist_s=1000.0, watch=False)
        m.wait_shards(1, 5)
        assert t.live == 8
        t0 = time.time()
        lease.close()
        while t.live and time.time() - t0 < 5:
            m.apply()
            time.sleep(0.02)
        assert t.live == 0 and not m.shards and t.tombstones == 8  # swept (K6), not deleted by an event
        assert time.time() - t0 < 1.0
        m.close()
    finally:
        c.Close()


def test_mirror_relist_catches_a_changed_record(tmp_path, ports, monkeypatch):
    """with no watch event for it, a record that CHANGED after it
    was applied (a ShardLease.update: a new generation's geometry) is caught by
    the re-list -- not only a key never applied -- and the mirror follows it."""
    monkeypatch.setenv("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    from ptype_amd import cluster as C
    from ptype_amd.mirror import RegistryMirror, ShardLease
    from ptype_amd.ops.table import RegistryTable

    pp, pc = ports(), ports()
    cfg = C.Config()
    cfg.service_name, cfg.node_name, cfg.port = "svc", "n0", ports()
    cfg.member = _member(C, 0, [pp], [pc], f"e0=http://127.0.0.1:{pp}", str(tmp_path))
    c = C.Join(C.background(), cfg, runtime=False)
    try:
        kv = c._c.registry.kv
        lease = ShardLease(kv, "svc", "x", 0, 1, 8)
        t = RegistryTable(256, device="cpu")
        m = RegistryMirror(t, kv, "svc", relist_s=0.2, watch=False)  # the re-list is the only follower
        m.wait_shards(1, 5)
        assert t.live == 8
        lease.update(count=24)  # same key, new record
        t0 = time.time()
        while t.live != 24 and time.time() - t0 < 5:
            m.apply()
            time.sleep(0.05)
        assert t.live == 24 and time.time() - t0 < 2.0, t.live
        m.close()
        lease.close()
    finally:
        c.Close()


def test_send_names_a_hosted_service():
    """A Send names its service: the runtime's own, or one co-hosted on its actors
    (host() / serve()); anything else is refused instead of silently routed."""
    import torch

    from ptype_amd.ops import batch as B
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY
    from ptype_amd.runtime import DeviceRuntime

    rt = DeviceRuntime(torch.device("cpu"), actors=16, service="calculator")
    rt.place_local()
    b = B.gen_requests(64, 16, METHOD_CALC_MULTIPLY, seed=3, device="cpu")
    v, st = rt.send("calculator", b)
    assert torch.equal(v, b.a0 * b.a1)
    with pytest.raises(ValueError, match="co-host"):
        rt.send("Prime", b)
    rt.host("Prime")
    v, _ = rt.send("Prime", b)
    assert torch.equal(v, b.a0 * b.a1)
    rt.close()


def test_join_world1_reforms_after_a_flagged_failure(tmp_path, ports, monkeypatch):
    """The CPU twin of test_elastic_gpu's Join case: gloo group formed by Join at
    world 1 (``form_group``), a generation flagged failed, the next Send
    re-forms generation 1 through the store and re-sends."""
    monkeypatch.setenv("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    from ptype_amd import cluster as C
    from ptype_amd.ops.batch import MsgBatch
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD, STATUS_OK

    pp, pc = ports(), ports()
    cfg = C.Config()
    cfg.service_name, cfg.node_name, cfg.port = "w1", "n0", ports()
    cfg.member = _member(C, 0, [pp], [pc], f"e0=http://127.0.0.1:{pp}", str(tmp_path))
    cfg.has_gpu = True
    cfg.gpu.cpu, cfg.gpu.world, cfg.gpu.form_group, cfg.gpu.actors, cfg.gpu.grace_s = True, 1, True, 64, 0.3
    srv = C.Serve(cfg.port, Host(), host="127.0.0.1")
    c = C.Join(C.background(), cfg)
    try:
        rt = c.runtime
        client = c.NewClient("w1", C.ConnConfig(retries=0))
        ids = torch.arange(rt.total_actors, dtype=torch.int32)
        add = MsgBatch(ids, torch.ones(ids.numel(), dtype=torch.int64), None, None, METHOD_COUNTER_ADD)
        assert bool((client.Send(add)[1] == STATUS_OK).all())
        rt.fail_generation("injected")
        mul = MsgBatch(ids, ids.to(torch.int64), torch.full((ids.numel(),), 3, dtype=torch.int64), None,
                       METHOD_CALC_MULTIPLY)
        val, st = client.Send(mul)
        assert bool((st == STATUS_OK).all()) and torch.equal(val, ids.to(torch.int64) * 3)
        assert bool((client.Send(add)[1] == STATUS_OK).all())
        assert rt.membership["gen"] == 1 and rt.recoveries == 1
        assert rt.state.unique().tolist() == [2] and rt.shard_lease.record["gen"] == 1
        rt.sync()
        assert len(rt.mirror.shards) == 1 and rt.table.live == rt.total_actors
        client.Close()
    finally:
        c.Close()
        srv.Close()


def test_native_dataplane_membership_on_cpu(tmp_path, ports, monkeypatch):
    """The compiled data plane's membership half (csrc/core/dataplane.cpp) without a
    GPU: live nodes from the registry's leases, wait_nodes, and settle -- bounded by
    its grace when nobody of the current members is gone, and the survivors in
    their old order once a member's registration ends (the next generation's
    proposal).  (form / ncclCommInitRank: tests/test_elastic_gpu.py.)"""
    monkeypatch.setenv("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    from ptype_amd import _core
    from ptype_amd import cluster as C

    if not _core.DataPlane.available():
        pytest.skip("RCCL / HIP entry points not loaded in this process")
    pp, pc, pa, pb = ports(), ports(), ports(), ports()
    cfg = C.Config()
    cfg.service_name, cfg.node_name, cfg.port = "dp", "a", pa
    cfg.member = _member(C, 0, [pp], [pc], f"e0=http://127.0.0.1:{pp}", str(tmp_path))
    c = C.Join(C.background(), cfg, runtime=False)
    other = None
    try:
        me, b = f"127.0.0.1:{pa}", f"127.0.0.1:{pb}"
        other = C.new_etcd_registry([f"http://127.0.0.1:{pc}"])
        other.Register(C.background(), "dp", "b", "127.0.0.1", pb)
        dp = _core.DataPlane(c._c, "dp", me, -1, 10.0)
        t0 = time.time()
        while sorted(dp.alive_nodes()) != sorted([me, b]) and time.time() - t0 < 10:
            time.sleep(0.05)
        assert sorted(dp.alive_nodes()) == sorted([me, b])
        assert dp.wait_nodes(2) == sorted([me, b])
        # nobody of the current members is gone: the proposal after the grace, unchanged
        t0 = time.time()
        assert dp.settle([b, me], 0.4) == [b, me]
        assert 0.35 < time.time() - t0 < 3.0
        # b's registration ends: the survivors, without waiting out a long grace
        other.close()
        other = None
        t0 = time.time()
        assert dp.settle([b, me], 15.0) == [me]
        assert time.time() - t0 < 8.0  # (the 2 s lease, or at once when the close revoked it)
        # a proposal that lost this member too still carries it
        assert dp.settle([b], 0.2) == [me]
    finally:
        if other is not None:
            other.close()
        c.Close()


def test_native_dataplane_rendezvous_converges_on_cpu(tmp_path, ports, monkeypatch):
    """The compiled rendezvous without a GPU: the first current record of a
    generation wins -- a member whose proposal differs adopts it, a member it
    leaves out learns it is excluded -- and the communicator step (hipSetDevice,
    ncclCommInitRank) is the only part left (it fails here for want of a device)."""
    monkeypatch.setenv("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    from ptype_amd import _core
    from ptype_amd import cluster as C

    if not _core.DataPlane.available():
        pytest.skip("RCCL / HIP entry points not loaded in this process")
    pp, pc, pa, pb = ports(), ports(), ports(), ports()
    cfg = C.Config()
    cfg.service_name, cfg.node_name, cfg.port = "rv", "a", pa
    cfg.member = _member(C, 0, [pp], [pc], f"e0=http://127.0.0.1:{pp}", str(tmp_path))
    c = C.Join(C.background(), cfg, runtime=False)
    other = C.new_etcd_registry([f"http://127.0.0.1:{pc}"])
    try:
        me, b = f"127.0.0.1:{pa}", f"127.0.0.1:{pb}"
        other.Register(C.background(), "rv", "b", "127.0.0.1", pb)
        da = _core.DataPlane(c._c, "rv", me, -1, 5.0)
        db = _core.DataPlane(c._c, "rv", b, -1, 5.0)
        da.wait_nodes(2)
        # a proposes [a] alone (its view: b is gone) and publishes generation 3's record
        with pytest.raises(RuntimeError, match="no device"):
            da.form(3, [me])
        # b, proposing [a, b], adopts the published record -- and is not in it
        with pytest.raises(RuntimeError, match="excluded"):
            db.form(3, [me, b])
        # a record for a later generation with both: b is rank 1 of it (reaches the device step)
        with pytest.raises(RuntimeError, match="no device"):
            da.form(4, [me, b])
        with pytest.raises(RuntimeError, match="no device"):
            db.form(4, [me, b])
        # a member outside its own proposal is refused at once
        with pytest.raises(RuntimeError, match="not in the proposal"):
            db.form(5, [me])
    finally:
        other.close()
        c.Close()

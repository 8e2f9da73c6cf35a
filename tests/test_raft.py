"""Raft control plane under multi-member scenarios (SURVEY C7, §7 hard part 1):
static bootstrap, leader failover, follower restart from the WAL, proposal
forwarding, snapshot shipping to a lagging learner.  All members run in this
process over loopback TCP, each with its own data dir."""
import threading
import time

import pytest

from ptype_amd import _core
from ptype_amd import cluster as C


def mk(name, ports, workdir, peers=None, state="new", snap=100000):
    pp, pc = ports(), ports()
    return C.member_config(name=name, dir=str(workdir / name), lpurls=[f"http://127.0.0.1:{pp}"],
                           apurls=[f"http://127.0.0.1:{pp}"], lcurls=[f"http://127.0.0.1:{pc}"],
                           acurls=[f"http://127.0.0.1:{pc}"], heartbeat_ms=20, election_ms=200,
                           cluster_state=state, unsafe_no_fsync=True, snapshot_count=snap)


def start_all(cfgs):
    ms = [_core.Member(c) for c in cfgs]
    ths = [threading.Thread(target=m.start) for m in ms]
    [t.start() for t in ths]
    [t.join() for t in ths]
    for m in ms:
        assert m.wait_ready(10000)
    return ms


def static_cluster(n, ports, workdir, snap=100000):
    cfgs = [mk(f"m{i}", ports, workdir, snap=snap) for i in range(n)]
    ic = ",".join(f"{c.name}={c.apurls[0]}" for c in cfgs)
    for c in cfgs:
        c.initial_cluster = ic
    return cfgs, start_all(cfgs)


def eps(cfg):
    return list(cfg.lcurls)


def wait_for(pred, timeout=10.0):
    t = time.time() + timeout
    while time.time() < t:
        if pred():
            return True
        time.sleep(0.02)
    return False


def test_static_bootstrap_replicates(tmp_path, ports):
    cfgs, ms = static_cluster(3, ports, tmp_path)
    try:
        leaders = {m.leader() for m in ms}
        assert len(leaders) == 1 and 0 not in leaders
        assert sorted(x.name for x in ms[0].member_list()) == ["m0", "m1", "m2"]
        # write through a follower: Raft forwards the proposal to the leader
        follower = [i for i, m in enumerate(ms) if m.id != ms[0].leader()][0]
        kv = _core.KvClient(eps(cfgs[follower]))
        kv.put("k", b"v1")
        for c in cfgs:
            k2 = _core.KvClient(eps(c))
            assert [x.value for x in k2.get("k").kvs] == [b"v1"]  # linearizable read everywhere
            k2.close()
        kv.close()
    finally:
        for m in ms:
            m.close()


def test_leader_failover_and_follower_restart(tmp_path, ports):
    cfgs, ms = static_cluster(3, ports, tmp_path)
    try:
        lid = ms[0].leader()
        li = [i for i, m in enumerate(ms) if m.id == lid][0]
        ms[li].close()
        alive = [i for i in range(3) if i != li]
        assert wait_for(lambda: ms[alive[0]].leader() not in (0, lid)), "no new leader elected"
        kv = _core.KvClient(eps(cfgs[alive[0]]))
        kv.put("after", b"failover")
        assert [x.value for x in kv.get("after").kvs] == [b"failover"]
        # restart the old leader on its data dir: it rejoins and catches up
        ms[li] = _core.Member(cfgs[li])
        ms[li].start()
        assert ms[li].wait_ready(10000)
        k3 = _core.KvClient(eps(cfgs[li]))
        o = _core.RangeOpts()
        o.serializable = True
        assert wait_for(lambda: [x.value for x in k3.get("after", o).kvs] == [b"failover"])
        k3.close()
        kv.close()
    finally:
        for m in ms:
            m.close()


def test_quorum_loss_blocks_writes(tmp_path, ports):
    cfgs, ms = static_cluster(3, ports, tmp_path)
    try:
        a, b, c = ms
        b.close()
        c.close()
        kv = _core.KvClient(eps(cfgs[0]))
        with pytest.raises((C.TimeoutError, C.PtypeError)):
            kv.put("x", b"y", 0)  # no quorum: the leader steps down (check-quorum), the write times out
        kv.close()
    finally:
        for m in ms:
            m.close()


def test_snapshot_catch_up_of_new_learner(tmp_path, ports):
    cfgs, ms = static_cluster(1, ports, tmp_path, snap=20)
    try:
        kv = _core.KvClient(eps(cfgs[0]))
        for i in range(120):  # several snapshots + log compaction
            kv.put(f"key{i:03d}", str(i).encode())
        new = mk("late", ports, tmp_path, state="existing")
        member, members = kv.member_add(list(new.lpurls), True)
        new.initial_cluster = ",".join([f"m0={cfgs[0].apurls[0]}", f"late={new.apurls[0]}"])
        late = _core.Member(new)
        late.start()
        assert late.wait_ready(10000)  # needs the snapshot: the log prefix was compacted
        o = _core.RangeOpts()
        o.serializable = True
        o.end = _core.prefix_range_end("key")
        k2 = _core.KvClient(eps(new))
        assert wait_for(lambda: k2.get("key", o).count == 120)
        assert late.is_learner()
        kv.member_promote(late.id)
        assert wait_for(lambda: not late.is_learner())
        k2.close()
        late.close()
        kv.close()
    finally:
        for m in ms:
            m.close()


def test_watch_on_follower_and_compaction(tmp_path, ports):
    cfgs, ms = static_cluster(3, ports, tmp_path)
    try:
        ctx = C.Context.with_cancel(None)
        kvf = _core.KvClient(eps(cfgs[2]))
        ch = kvf.watch(ctx, "w/", _core.prefix_range_end("w/"))
        kvl = _core.KvClient(eps(cfgs[0]))
        r1 = kvl.put("w/a", b"1")
        kvl.put("w/b", b"2")
        kvl.delete("w/a")
        evs = []
        wait_for(lambda: (evs.extend((ch.recv(0.05) or _Empty()).events) or len(evs) >= 3), 5)
        assert [(e.type, e.kv.key) for e in evs[:3]] == [("PUT", "w/a"), ("PUT", "w/b"), ("DELETE", "w/a")]
        kvl.compact(r1)
        o = _core.RangeOpts()
        o.rev = r1 - 1
        with pytest.raises(C.PtypeError, match="compacted"):
            kvl.get("w/a", o)
        ctx.cancel()
        kvf.close()
        kvl.close()
    finally:
        for m in ms:
            m.close()


class _Empty:
    events = []


def test_linearizable_reads_use_read_index(tmp_path, ports):
    """A linearizable Get is a ReadIndex round (leader commit index confirmed by a
    quorum of heartbeat acks), not a log entry: reads leave the log untouched, and
    a read on any member -- follower included -- sees every write acknowledged
    before it started (reference: etcd's default linearizable Range,
    cluster/store.go:38-53)."""
    cfgs, ms = static_cluster(3, ports, tmp_path)
    try:
        leader_id = ms[0].leader()
        follower = [i for i, m in enumerate(ms) if m.id != leader_id][0]
        leader = [i for i, m in enumerate(ms) if m.id == leader_id][0]
        w = _core.KvClient(eps(cfgs[leader]))
        r = _core.KvClient(eps(cfgs[follower]))
        w.put("x", b"0")
        assert wait_for(lambda: ms[follower].status().applied == ms[leader].status().applied)
        before = ms[leader].status().commit
        for i in range(1, 40):
            w.put("x", str(i).encode())  # acknowledged by the leader ...
            assert [kv.value for kv in r.get("x").kvs] == [str(i).encode()]  # ... visible on the follower
        after_writes = ms[leader].status().commit
        assert after_writes - before == 39  # one entry per put, none per get
        for _ in range(50):
            r.get("x")
        time.sleep(0.1)
        assert ms[leader].status().commit == after_writes  # 50 linearizable reads: no log growth
        assert ms[follower].reads_served >= 89
        w.close()
        r.close()
    finally:
        for m in ms:
            m.close()

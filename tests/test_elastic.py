"""Data-plane rank failure and recovery, on CPU with gloo.

Three processes, each a control-plane member + a data-plane rank hosting 64
actors.  After one batch, one process dies abruptly (``os._exit``: no cleanup,
its Raft member and registry lease die with it).  The survivors' next ``Send``
fails inside the collective, they abort the group, wait for the dead node's
lease to expire, form generation 1 through the replicated store, re-home the
dead rank's actors and re-send: every actor is reachable again, actors of live
ranks kept their state, and the adopted actors resumed from the buddy replica
taken before the crash (``replicate``), not from zero.
"""
import os

import pytest
import torch
import torch.multiprocessing as mp

from ptype_amd.parallel.elastic import buddy, ring_placement


def test_ring_placement():
    n = ["a", "b", "c", "d"]
    assert ring_placement(n, n) == {"a": [0], "b": [1], "c": [2], "d": [3]}
    assert ring_placement(n, ["a", "b", "d"]) == {"a": [0], "b": [1], "d": [3, 2]}
    assert ring_placement(n, ["a", "c"]) == {"a": [0, 3], "c": [2, 1]}
    assert ring_placement(n, ["d"]) == {"d": [3, 0, 1, 2]}
    # the buddy of a node is the adopter of everything it hosts
    for alive in (n, ["a", "b", "d"], ["a", "c"]):
        own = ring_placement(n, alive)
        for h in alive:
            rest = [x for x in alive if x != h]  # h dies
            assert buddy(n, alive, h) in rest
            assert set(own[h]) <= set(ring_placement(n, rest)[buddy(n, alive, h)])
    assert buddy(n, ["c"], "c") == "c"


def _worker(i, pp, pc, sp, crash, q):
    os.environ["PTYPE_ADVERTISE_ADDR"] = "127.0.0.1"
    import tempfile

    from ptype_amd import cluster as C
    from ptype_amd.ops.batch import MsgBatch
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD, STATUS_OK
    from ptype_amd.parallel.elastic import ElasticDataPlane

    try:
        ic = ",".join(f"e{j}=http://127.0.0.1:{pp[j]}" for j in range(3))
        cfg = C.Config()
        cfg.service_name, cfg.node_name, cfg.port = "dp", f"n{i}", sp[i]
        cfg.member = C.member_config(name=f"e{i}", dir=tempfile.mkdtemp(prefix=f"el{i}_"),
                                     lpurls=[f"http://127.0.0.1:{pp[i]}"], apurls=[f"http://127.0.0.1:{pp[i]}"],
                                     lcurls=[f"http://127.0.0.1:{pc[i]}"], acurls=[f"http://127.0.0.1:{pc[i]}"],
                                     initial_cluster=ic, heartbeat_ms=20, election_ms=200, unsafe_no_fsync=True)
        c = C.Join(C.background(), cfg)
        dp = ElasticDataPlane(c, "dp", world=3, per_rank=64, timeout_s=5.0, grace_s=10.0)
        dp.start()
        n = dp.total_actors
        ids = torch.arange(n, dtype=torch.int32)
        add = MsgBatch(ids, torch.ones(n, dtype=torch.int64), None, None, METHOD_COUNTER_ADD)
        _, st = dp.send_resilient(add)
        ok1 = bool((st == STATUS_OK).all()) and bool((dp.state == 3).all())
        dp.replicate()  # every block now has a copy on its buddy
        if dp.me == dp.nodes0[crash]:
            os._exit(0)  # crash: no group teardown, no lease revoke, member gone
        mul = MsgBatch(ids, ids.to(torch.int64), torch.full((n,), 7, dtype=torch.int64), None, METHOD_CALC_MULTIPLY)
        val, st = dp.send_resilient(mul)
        ok2 = bool((st == STATUS_OK).all()) and torch.equal(val, ids.to(torch.int64) * 7)
        _, st = dp.send_resilient(add)
        ok3 = bool((st == STATUS_OK).all())
        # own block: 3 + 2 increments; adopted block (if any): its replica (3) + 2 increments
        P = dp.per_rank
        own = bool((dp.state[:P] == 5).all())
        adopted = [int(x) for x in dp.state[P:].unique().tolist()]
        q.put((dp.me, ok1, ok2, ok3, own, adopted, dp.restored, len(dp.members), dp.recoveries, dp.blocks))
        dp.close()
        c.Close()
    except Exception as e:
        import traceback

        try:
            st = c._c.member_status()
            diag = f"member id={st.id} leader={st.leader} term={st.term} commit={st.commit} applied={st.applied}"
        except Exception as e2:
            diag = repr(e2)
        q.put(("error", repr(e), diag, traceback.format_exc()[-1500:]))


@pytest.mark.timeout(180)
def test_rank_failure_recovery():
    from conftest import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pp, pc, sp = ([free_port() for _ in range(3)] for _ in range(3))
    crash = 1
    procs = [ctx.Process(target=_worker, args=(i, pp, pc, sp, crash, q)) for i in range(3)]
    [p.start() for p in procs]
    res = [q.get(timeout=150) for _ in range(2)]
    [p.join(30) for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    errors = [r for r in res if r[0] == "error"]
    assert not errors, "\n".join("\n".join(map(str, r)) for r in errors)
    for me, ok1, ok2, ok3, own, adopted, restored, world, recoveries, blocks in res:
        assert ok1 and ok2 and ok3 and own, (me, ok1, ok2, ok3, own)
        assert world == 2 and recoveries == 1
        if len(blocks) > 1:
            assert blocks[1] == crash and restored == [crash] and adopted == [5], (blocks, restored, adopted)
    assert sorted(len(r[-1]) for r in res) == [1, 2]  # exactly one survivor adopted the dead rank

"""Rank failure on the NATIVE GPU data plane, across processes.

Three processes on one GPU, each ``Join`` with a ``gpu:`` section (``world: 3``,
``comm: ipc``): the compiled DataPlane (csrc/core/dataplane.cpp) forms the group
through the replicated store with the IpcComm transport (shared-memory segments
that every rank maps and registers with HIP, csrc/hip/ipc_comm.hpp) -- the same
form / abort / settle / next-generation code as RCCL, and no torch process
group at all.  One node dies without cleanup after the first
round; the survivors' ``Client.Send`` sees the dead peer at the comm's timeout,
the DataPlane aborts the generation, waits for the lease-driven membership,
forms generation 1 through the store and hands back the ring adoption; the
adopter resumes the dead rank's actors from the buddy replica --
messages of lost actors answer STATUS_RANK_LOST when re-sends are off, and are
answered by the adopter afterwards.  The CPU twin is
tests/test_dataplane.py::test_join_send_survives_a_dead_rank.
"""
import os

import pytest
import torch
import torch.multiprocessing as mp

from conftest import free_port

pytestmark = pytest.mark.gpu


class Host:
    def Ping(self, x):
        return x


def _survivor(i, pp, pc, sp, tmp, crash, q):
    os.environ["PTYPE_ADVERTISE_ADDR"] = "127.0.0.1"
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    from ptype_amd import cluster as C
    from ptype_amd.ops.batch import MsgBatch
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD, STATUS_OK, STATUS_RANK_LOST

    c = None
    try:
        ic = ",".join(f"e{j}=http://127.0.0.1:{pp[j]}" for j in range(3))
        cfg = C.Config()
        cfg.service_name, cfg.node_name, cfg.port = "calc", f"n{i}", sp[i]
        cfg.member = C.member_config(name=f"e{i}", dir=os.path.join(tmp, f"m{i}"),
                                     lpurls=[f"http://127.0.0.1:{pp[i]}"], apurls=[f"http://127.0.0.1:{pp[i]}"],
                                     lcurls=[f"http://127.0.0.1:{pc[i]}"], acurls=[f"http://127.0.0.1:{pc[i]}"],
                                     initial_cluster=ic, heartbeat_ms=20, election_ms=200, unsafe_no_fsync=True)
        cfg.has_gpu = True
        g = cfg.gpu
        g.device, g.world, g.actors, g.max_batch, g.comm = 0, 3, 64, 8192, "ipc"
        g.group_timeout_s, g.grace_s, g.send_timeout_s = 4.0, 10.0, 0.0
        srv = C.Serve(sp[i], Host(), host="127.0.0.1")
        c = C.Join(C.background(), cfg)
        rt = c.runtime
        client = c.NewClient("calc", C.ConnConfig(retries=0, allow_local=False))
        n = rt.total_actors
        dev = rt.device
        ids = torch.arange(n, dtype=torch.int32, device=dev)
        add = MsgBatch(ids, torch.ones(n, dtype=torch.int64, device=dev), None, None, METHOD_COUNTER_ADD)
        _, st = client.Send(add)
        import torch.distributed as dist

        ok1 = bool((st == STATUS_OK).all()) and rt.exchange.ipc is not None
        ok1 = ok1 and type(rt.group).__name__ == "NativeGroup" and rt.group.transport == "ipc"
        ok1 = ok1 and not dist.is_initialized()  # no torch process group anywhere
        rt.replicate()  # every block has a copy on its buddy (the node that adopts it)
        me = rt.membership["me"]
        dead = rt.membership["nodes0"][crash]
        if me == dead:
            os._exit(0)  # crash: no group teardown, no lease revoke, its Raft member gone
        a = ids.to(torch.int64) + 100 * i
        mul = MsgBatch(ids, a, torch.full((n,), 7, dtype=torch.int64, device=dev), None, METHOD_CALC_MULTIPLY)
        val, st = client.Send(mul, resend_overflow=False)
        lost = (ids % 3) == crash
        ok_lost = bool((st[lost] == STATUS_RANK_LOST).all()) and bool((st[~lost] == STATUS_OK).all()) \
            and torch.equal(val[~lost], a[~lost] * 7)
        val, st = client.Send(mul)  # re-sent: the adopter answers now
        ok2 = ok_lost and bool((st == STATUS_OK).all()) and torch.equal(val, a * 7)
        _, st = client.Send(add)
        ok3 = bool((st == STATUS_OK).all())
        rt.group.barrier()
        P = rt.actors
        own = sorted(int(x) for x in rt.state[:P].unique().tolist())
        adopted = sorted(int(x) for x in rt.state[P:].unique().tolist())
        q.put((me, dead, ok1, ok2, ok3, own, adopted, rt.restored, rt.world, rt.recoveries, rt.blocks,
               rt.membership["gen"], rt.exchange.ipc is not None))
        rt.group.barrier()
        client.Close()
        srv.Close()
        c.Close()
    except Exception as e:
        import traceback

        q.put(("error", i, repr(e), traceback.format_exc()[-2500:]))
        if c is not None:
            c.Close()


@pytest.mark.timeout(300)
def test_native_ipc_data_plane_survives_a_killed_rank(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pp, pc, sp = ([free_port() for _ in range(3)] for _ in range(3))
    crash = 1
    procs = [ctx.Process(target=_survivor, args=(i, pp, pc, sp, str(tmp_path), crash, q)) for i in range(3)]
    [p.start() for p in procs]
    try:
        res = [q.get(timeout=240) for _ in range(2)]
    finally:
        [p.join(30) for p in procs]
        for p in procs:
            if p.is_alive():
                p.kill()
    errors = [r for r in res if r[0] == "error"]
    assert not errors, "\n".join("\n".join(map(str, r)) for r in errors)
    for me, dead, ok1, ok2, ok3, own, adopted, restored, world, recov, blocks, gen, ipc in res:
        assert ok1 and ok2 and ok3 and ipc, (me, ok1, ok2, ok3, ipc)
        assert world == 2 and recov == 1 and gen == 1, (world, recov, gen)
        assert own == [5], own  # 3 adds before the crash (one per rank), 2 after (two survivors)
        if len(blocks) > 1:  # the adopter: the dead rank's actors resumed from the replica (3) + 2
            assert blocks[1] == crash and restored == [crash] and adopted == [5], (blocks, restored, adopted)
    assert sorted(len(r[10]) for r in res) == [1, 2]  # exactly one survivor adopted the dead rank

"""Exchange-epoch engine across processes (CPU, gloo, world size 2 and 3).

The same ActorExchange code drives RCCL on MI355X; here the collectives run on
gloo and the kernels on their plain-PyTorch references, so the distributed
logic (bucketing, equal-split all-to-all of epoch slots, reply routing, overflow
re-send, stateful actors) is covered without a GPU."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ptype_amd.ops import batch as B
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD, STATUS_OK
from ptype_amd.ops.table import RegistryTable, actor_keys
from ptype_amd.parallel.exchange import ActorExchange


def _worker(rank, world, port, scenario, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        per_rank = 64
        n_actors = per_rank * world
        table = RegistryTable(4 * n_actors, device="cpu")
        ids = torch.arange(n_actors)
        table.upsert(actor_keys(ids), (ids % world).to(torch.int32), (ids // world).to(torch.int32))
        state = torch.zeros(per_rank, dtype=torch.int64)
        if scenario == "multiply":
            M = 3000 + 117 * rank  # uneven batch sizes per rank
            req = B.gen_requests(M, n_actors, METHOD_CALC_MULTIPLY, seed=rank + 1, device="cpu")
            ex = ActorExchange(table, M, chunks=3, state=state)
            val, st = ex.send(req)
            ok = bool((st == STATUS_OK).all()) and torch.equal(val, req.a0 * req.a1)
            q.put((rank, ok, int(M)))
        elif scenario == "overflow":
            M = 2000
            # every message of rank r goes to actors hosted on rank 0 -> bucket 0 overflows
            actors = (torch.arange(M) * world % n_actors).to(torch.int32)
            req = B.MsgBatch(actors, torch.arange(M, dtype=torch.int64), torch.full((M,), 3, dtype=torch.int64), None,
                             METHOD_CALC_MULTIPLY)
            ex = ActorExchange(table, M, chunks=1, state=state)
            ex.C = 512  # force a tiny capacity: 4 epochs needed
            from ptype_amd.parallel.exchange import _ChunkBufs

            ex.bufs = [_ChunkBufs(world, ex.C, ex.max_chunk, ex.device)]
            val, st = ex.send_all(req)
            ok = bool((st == STATUS_OK).all()) and torch.equal(val, torch.arange(M) * 3)
            q.put((rank, ok, M))
        elif scenario == "counter":
            M = 1000
            actors = (torch.arange(M) % n_actors).to(torch.int32)
            req = B.MsgBatch(actors, torch.ones(M, dtype=torch.int64), None, None, METHOD_COUNTER_ADD)
            ex = ActorExchange(table, M, chunks=2, state=state)
            val, st = ex.send(req)
            dist.barrier()
            total = state.sum()
            dist.all_reduce(total)
            ok = bool((st == STATUS_OK).all()) and int(total) == M * world
            q.put((rank, ok, int(state.sum())))
    except Exception as e:  # surface worker failures to the parent
        q.put((rank, False, repr(e)))
    finally:
        dist.destroy_process_group()


def _run(world, scenario):
    from conftest import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, scenario, q)) for r in range(world)]
    [p.start() for p in procs]
    res = [q.get(timeout=60) for _ in range(world)]
    [p.join(60) for p in procs]
    return sorted(res)


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_multiply_across_ranks(world):
    res = _run(world, "multiply")
    assert all(ok for _, ok, _ in res), res


def test_exchange_overflow_resend():
    res = _run(2, "overflow")
    assert all(ok for _, ok, _ in res), res


def test_exchange_stateful_actors():
    res = _run(2, "counter")
    assert all(ok for _, ok, _ in res), res

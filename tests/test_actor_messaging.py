"""Actor-to-actor messaging on the device: handlers emit into an
HBM outbox, ``ActorExchange.pump`` routes the emitted messages epoch after epoch
until every outbox is empty.  Token ring: T tokens each make H hops of stride s
over n actors; every actor must count exactly the visits a plain simulation
predicts.  CPU (reference dispatch, gloo for 2 ranks) and GPU."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ptype_amd.ops import batch as B
from ptype_amd.ops.outbox import DeviceOutbox
from ptype_amd.ops.records import METHOD_FORWARD
from ptype_amd.ops.table import RegistryTable, actor_keys
from ptype_amd.parallel.exchange import ActorExchange


def _expected_visits(n, starts, hops, stride):
    v = torch.zeros(n, dtype=torch.int64)
    for s in starts:
        a = s
        for _ in range(hops + 1):
            v[a] += 1
            a = (a + stride) % n
    return v


def _tokens(n, starts, hops, stride, device):
    starts = torch.as_tensor(starts, dtype=torch.int64)
    T = starts.numel()
    nxt = (starts + stride) % n
    return B.MsgBatch(starts.to(torch.int32).to(device), nxt.to(device), torch.full((T,), hops, dtype=torch.int64,
                                                                                      device=device),
                      torch.full((T,), stride | (n << 32), dtype=torch.int64, device=device), METHOD_FORWARD)


def _ring(device, world=1, rank=0, n_per=64, T=20, hops=7, stride=5):
    n = n_per * world
    table = RegistryTable(4 * n, device=device)
    ids = torch.arange(n, dtype=torch.int64)
    table.upsert(actor_keys(ids), (ids % world).to(torch.int32), (ids // world).to(torch.int32))
    state = torch.zeros(n_per, dtype=torch.int64, device=device)
    cap = max(4096, T)
    ex = ActorExchange(table, cap, chunks=2, state=state)
    starts = [(rank * 131 + 17 * t) % n for t in range(T)]
    outbox = DeviceOutbox(cap, device=device)
    epochs, delivered = ex.pump(outbox, initial=_tokens(n, starts, hops, stride, device))
    return ex, state, starts, epochs, delivered, outbox, n


def test_token_ring_reference_single_rank():
    ex, state, starts, epochs, delivered, outbox, n = _ring("cpu")
    assert epochs == 7 and delivered == 20 * 8 and outbox.dropped == 0
    assert torch.equal(state, _expected_visits(n, starts, 7, 5))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ex, state, starts, epochs, delivered, outbox, n = _ring("cpu", world, rank)
        all_starts = [None] * world
        dist.all_gather_object(all_starts, starts)
        exp = _expected_visits(n, [s for ss in all_starts for s in ss], 7, 5)
        mine = exp[torch.arange(n) % world == rank]  # actor a -> rank a % world, mailbox a // world
        q.put((rank, bool(torch.equal(state, mine)), epochs))
    except Exception as e:
        q.put((rank, False, repr(e)))
    finally:
        dist.destroy_process_group()


def test_token_ring_across_ranks():
    from conftest import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    res = sorted(q.get(timeout=120) for _ in range(2))
    [p.join(60) for p in ps]
    assert all(ok for _, ok, _ in res), res
    assert all(e == 7 for _, _, e in res)


@pytest.mark.gpu
@pytest.mark.parametrize("pump", ["graph", "eager", "host"])
def test_token_ring_on_device(pump, monkeypatch):
    """``graph`` / ``eager``: epochs read their length from the outbox bank's
    device counter (one host check per 8 epochs; groups after the first replayed
    from a hipGraph, or launched one by one); ``host``: the host reads every
    epoch's count."""
    monkeypatch.setenv("PTYPE_TUNE", "device_pump=" + ("0" if pump == "host" else "1") + ",pump_graph="
                       + ("1" if pump == "graph" else "0"))
    n_per, T, hops, stride = 100_000, 50_000, 20, 7919
    ex, state, starts, epochs, delivered, outbox, n = _ring("cuda", 1, 0, n_per, T, hops, stride)
    torch.cuda.synchronize()
    assert epochs == hops and delivered == T * (hops + 1) and outbox.dropped == 0
    assert torch.equal(state.cpu(), _expected_visits(n, starts, hops, stride))


@pytest.mark.gpu
def test_outbox_overflow_counts_drops():
    n = 1000
    table = RegistryTable(4 * n, device="cuda")
    ids = torch.arange(n, dtype=torch.int64)
    table.upsert(actor_keys(ids), torch.zeros(n, dtype=torch.int32), ids.to(torch.int32))
    state = torch.zeros(n, dtype=torch.int64, device="cuda")
    ex = ActorExchange(table, 4096, state=state)
    outbox = DeviceOutbox(100, device="cuda")
    ex.outbox = outbox
    ex.send(_tokens(n, list(range(300)), 1, 1, "cuda"))
    torch.cuda.synchronize()
    assert outbox.pending() == 100 and outbox.dropped == 200

"""One rank of a multi-PROCESS data-plane test on one GPU (tests/test_ipc_comm_gpu.py).

Usage: python _ipc_worker.py <scenario> <rank> <world> <port>.  Every rank joins a
gloo group (the host side: segment names, host agreements, result gathering)
and drives the native engines' collectives through an IpcComm on cuda:0
(csrc/hip/ipc_comm.hpp: shared-memory segments every rank maps).  Rank 0
prints one ``RESULT {json}`` line; a failed check raises (non-zero exit)."""
import json
import os
import signal
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ptype_amd.ops import batch as B  # noqa: E402
from ptype_amd.ops import hip  # noqa: E402
from ptype_amd.ops.records import (METHOD_CALC_MULTIPLY, METHOD_SEQ_FOLD, STATUS_NOT_DELIVERED,  # noqa: E402
                                   STATUS_OK)
from ptype_amd.ops.table import RegistryTable, actor_keys  # noqa: E402
from ptype_amd.parallel.exchange import ActorExchange, ipc_group_comm  # noqa: E402

DEV = torch.device("cuda", 0)


def table(n, R, seed=99):
    t = RegistryTable(2 * n, device=DEV)
    ids = torch.arange(n)
    slot = torch.randperm(n, generator=torch.Generator().manual_seed(seed))  # random placement: routes read the mirror
    t.upsert(actor_keys(ids), (slot % R).to(torch.int32), (slot // R).to(torch.int32))
    t.enable_directory(n)
    return t, slot


def raw(rank, R):
    """Equal-split all-to-all, exact-prefix all-to-allv and all-reduce(MAX) through
    IpcComm, every word checked, over ops that reuse the inboxes."""
    cap = 1 << 16
    c = ipc_group_comm(None, DEV, cap, 20.0)
    s = torch.cuda.current_stream().cuda_stream
    n = cap // 4
    for op in range(12):
        src = torch.empty(R, n, dtype=torch.int32, device=DEV)
        for q in range(R):  # word j of region q from rank r: (op, r, q, j)
            src[q] = op * 1_000_000 + rank * 10_000 + q * 1000 + torch.arange(n, device=DEV) % 997
        dst = torch.full((R, n), -1, dtype=torch.int32, device=DEV)
        c.alltoall(src.data_ptr(), dst.data_ptr(), n * 4, s)
        torch.cuda.synchronize()
        for q in range(R):
            want = op * 1_000_000 + q * 10_000 + rank * 1000 + torch.arange(n, device=DEV) % 997
            assert torch.equal(dst[q], want), (op, q)
        v = torch.tensor([rank * 7 + op, 100 - rank, op], dtype=torch.int64, device=DEV)
        c.allreduce_max(v.data_ptr(), 3, s)
        torch.cuda.synchronize()
        assert v.tolist() == [(R - 1) * 7 + op, 100, op], v.tolist()
    assert not c.failed and c.ops == 24
    return {"ops": int(c.ops)}


def sorted_calc(rank, R):
    """The sorted exchange (N > 1 mailbox delivery) across processes: exact
    calculator replies from Send 0 (start-up layout) through Send 6 (agreed),
    the overflow count read from the agreement, Join's default delivery "auto"
    on the same engine, then skewed traffic through send_all."""
    n, M = 16384, 120_000
    tab, _ = table(n, R)
    st = torch.zeros(n // R + 1, dtype=torch.int64, device=DEV)
    out = {}
    for delivery in ("mailbox", "auto"):
        ex = ActorExchange(tab, M, chunks=2, state=st, delivery=delivery, mailbox_ordered=False, comm="ipc",
                           comm_timeout_s=30.0)
        wires = []
        for k in range(7):
            req = B.gen_requests(M - 1111 * rank, n, METHOD_CALC_MULTIPLY, seed=40 + 7 * rank + k, device=DEV)
            v, sts = ex.send(req)
            torch.cuda.synchronize()
            assert bool((sts == STATUS_OK).all()), (delivery, k, int((sts != STATUS_OK).sum()))
            assert torch.equal(v, req.a0 * req.a1), (delivery, k)
            assert int(ex._sorted.last_overflow()) == 0
            wires.append(dict(ex.last_wire))
        assert wires[0]["engine"] == "sorted" and not wires[0]["agreed"] and wires[0]["S"] == 8
        assert wires[2]["agreed"] and wires[6]["agreed"] and wires[6]["S"] <= 2 and wires[6]["vb"] == 4
        out[delivery] = {"C": int(wires[6]["C"]), "S": int(wires[6]["S"])}
        assert ex.stats().failed == 0
    # skew: Zipf(1.1) actor popularity -- send_all re-sends what the start-up capacity could not hold
    ex = ActorExchange(tab, M, chunks=2, state=st, delivery="mailbox", mailbox_ordered=False, comm="ipc")
    rounds = []
    for k in range(6):
        req = B.gen_zipf_requests(M, n, 1.1, seed=900 + 13 * rank + k, device=DEV)
        before = ex.counters.resends
        v, sts = ex.send_all(req)
        torch.cuda.synchronize()
        assert bool((sts == STATUS_OK).all()) and torch.equal(v, req.a0 * req.a1), k
        rounds.append(ex.counters.resends - before)
    assert sum(rounds[3:]) == 0, rounds  # once agreements size the regions: no re-send rounds
    out["zipf_resend_rounds"] = rounds
    return out


def sorted_fold(rank, R):
    """Ordered SeqFold traffic from every process to every process's actors: the
    replies gathered on rank 0 chain every actor's state exactly once, and each
    (sender, actor) pair ran in message order."""
    from ptype_amd.ops.mailbox import audit_fold

    n, M = 4096, 50_000
    tab, slot = table(n, R)
    s0 = torch.randint(0, 1 << 30, (n // R + 1,), dtype=torch.int64, generator=torch.Generator().manual_seed(rank))
    st = s0.to(DEV)
    ex = ActorExchange(tab, M, chunks=2, state=st, delivery="mailbox", comm="ipc")
    mine = []
    for k in range(3):
        g = torch.Generator().manual_seed(500 + 10 * rank + k)
        req = B.MsgBatch(torch.randint(0, n, (M,), generator=g, dtype=torch.int32).to(DEV),
                         torch.randint(-(1 << 20), 1 << 20, (M,), generator=g, dtype=torch.int64).to(DEV),
                         None, None, METHOD_SEQ_FOLD)
        v, sts = ex.send_all(req)
        torch.cuda.synchronize()
        mine.append((req.actor.cpu().long(), req.a0.cpu(), v.cpu(), sts.cpu()))
    parts = [None] * R
    dist.all_gather_object(parts, {"sends": mine, "before": s0, "after": st.cpu()})
    if rank != 0:
        return {}
    P = n // R + 1
    key_of = lambda a: (slot[a] % R) * P + slot[a] // R  # noqa: E731
    before = torch.cat([p["before"] for p in parts])
    after = torch.cat([p["after"] for p in parts])
    cols = [torch.cat([torch.cat([snd[j] for snd in p["sends"]]) for p in parts]) for j in range(4)]
    ok, order = audit_fold(key_of(cols[0]), cols[1], cols[2], cols[3], before, after)
    assert ok, order
    sizes = [sum(len(snd[0]) for snd in p["sends"]) for p in parts]
    bounds = torch.cumsum(torch.tensor([0] + sizes), 0)
    for x, seq in list(order.items())[:512]:
        for r in range(R):
            m = [i for i in seq if bounds[r] <= i < bounds[r + 1]]
            assert m == sorted(m), f"actor {x}: sender {r}'s messages out of order"
    return {"messages": int(bounds[-1]), "actors": len(order)}


def sorted_fold_defer(rank, R):
    """VERDICT r5 #2 / ADVICE r5: ordered SeqFold Sends through send_all(defer=True)
    with Zipf-skewed actors (the start-up capacity overflows: re-send rounds) and
    one Send whose arguments outgrow the agreed widths (null records: the FIFO
    fix-up overflows the rest of their buckets).  An ordered batch is never
    deferred -- its overflowed suffix runs before the next Send -- so across ALL
    Sends every (sender, actor) pair runs in message order, exactly once."""
    from ptype_amd.ops.mailbox import audit_fold

    n, M, K = 4096, 60_000, 7
    tab, slot = table(n, R)
    s0 = torch.randint(0, 1 << 30, (n // R + 1,), dtype=torch.int64, generator=torch.Generator().manual_seed(rank))
    st = s0.to(DEV)
    ex = ActorExchange(tab, M, chunks=2, state=st, delivery="mailbox", comm="ipc", comm_timeout_s=30.0)
    mine, rounds = [], []
    for k in range(K):
        actor = B.zipf_actors(M, n, 1.1, 1000 + 31 * rank + k, DEV)
        g = torch.Generator().manual_seed(2000 + 10 * rank + k)
        a0 = torch.randint(-(1 << 14), 1 << 14, (M,), generator=g, dtype=torch.int64)
        if k == 4:  # wider than the layout agreed from Send 2: null records + the bucket fix-up
            a0[::501] = (1 << 45) + k
        req = B.MsgBatch(actor.to(torch.int32), a0.to(DEV), None, None, METHOD_SEQ_FOLD)
        r0 = ex.counters.resends
        v, sts = ex.send_all(req, defer=True)
        assert not ex._deferred, "an ordered Send was deferred"
        rounds.append(ex.counters.resends - r0)
        mine.append((actor.cpu().long(), a0, v.cpu(), sts.cpu()))
    ex.flush()
    torch.cuda.synchronize()
    parts = [None] * R
    dist.all_gather_object(parts, {"sends": mine, "before": s0, "after": st.cpu(), "rounds": rounds})
    if rank != 0:
        return {}
    P = n // R + 1
    key_of = lambda a: (slot[a] % R) * P + slot[a] // R  # noqa: E731
    before = torch.cat([p["before"] for p in parts])
    after = torch.cat([p["after"] for p in parts])
    cols = [torch.cat([torch.cat([snd[j] for snd in p["sends"]]) for p in parts]) for j in range(4)]
    ok, order = audit_fold(key_of(cols[0]), cols[1], cols[2], cols[3], before, after)
    assert ok, order
    sizes = [sum(len(snd[0]) for snd in p["sends"]) for p in parts]
    bounds = torch.cumsum(torch.tensor([0] + sizes), 0).tolist()
    bad = 0
    for x, seq in order.items():  # indices are Send-major per sender: message order across Sends
        for r in range(R):
            m = [i for i in seq if bounds[r] <= i < bounds[r + 1]]
            bad += m != sorted(m)
    assert bad == 0, f"{bad} (sender, actor) pairs ran out of message order"
    return {"messages": int(bounds[-1]), "actors": len(order), "rounds": [p["rounds"] for p in parts]}


def sorted_defer(rank, R):
    """send_all(defer=True) across processes: no host wait on the
    current Send -- Send k's overflow count is read just before Send k + 2 (its
    agreement, which Send k + 2 waits for anyway) -- then flush(); every reply
    exact, skewed start-up Sends included (their overflow re-sent late, into the
    same output tensors).  Host time per Send reported without the backpressure
    wait for Send k - 2's agreement."""
    n, M = 16384, 120_000
    tab, _ = table(n, R)
    st = torch.zeros(n // R + 1, dtype=torch.int64, device=DEV)
    ex = ActorExchange(tab, M, chunks=2, state=st, delivery="mailbox", mailbox_ordered=False, comm="ipc",
                       comm_timeout_s=30.0)
    outs, host = [], []
    K = 12
    for k in range(K):
        # Zipf-skewed early Sends overflow the start-up capacity; uniform later ones fit
        req = (B.gen_zipf_requests(M, n, 1.1, seed=300 + 17 * rank + k, device=DEV) if k < 3 else
               B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=700 + 7 * rank + k, device=DEV))
        t = time.perf_counter()
        v, sts = ex.send_all(req, defer=True)
        host.append(time.perf_counter() - t)
        outs.append((req, v, sts))
        # deferred: only Sends at least two old were resolved (their agreement adopted already)
        assert all(d[0] <= ex._sorted.sends - 2 for d in ex._deferred) or len(ex._deferred) <= 2
    prof = ex._sorted.host_profile()
    waits_before_flush = int(prof["overflow_waits"])
    ex.flush()
    torch.cuda.synchronize()
    for k, (req, v, sts) in enumerate(outs):
        assert bool((sts == STATUS_OK).all()), (k, int((sts != STATUS_OK).sum()))
        assert torch.equal(v, req.a0 * req.a1), k
    rounds_skewed = int(ex.counters.resends)
    # steady state (uniform traffic, agreed capacity): the only overflow reads are of
    # Sends two Sends old -- none of the current Send -- and no re-send round runs
    w0, r0, outs = int(ex._sorted.host_profile()["overflow_waits"]), int(ex.counters.resends), []
    for k in range(K):
        req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=900 + 7 * rank + k, device=DEV)
        outs.append((req,) + tuple(ex.send_all(req, defer=True)))
    steady_waits = int(ex._sorted.host_profile()["overflow_waits"]) - w0
    ex.flush()
    torch.cuda.synchronize()
    for k, (req, v, sts) in enumerate(outs):
        assert bool((sts == STATUS_OK).all()) and torch.equal(v, req.a0 * req.a1), k
    prof = ex._sorted.host_profile()
    sends = int(prof["sends"])
    return {"resend_rounds": rounds_skewed, "steady_resend_rounds": int(ex.counters.resends) - r0,
            "steady_overflow_waits": steady_waits, "overflow_waits_before_flush": waits_before_flush,
            "deferred_sends": K, "host_us_per_send_all": sorted(host)[len(host) // 2] * 1e6,
            "host_us_per_native_send": (prof["total_ns"] - prof["spec_wait_ns"]) / max(sends, 1) / 1e3,
            "backpressure_us_per_send": prof["spec_wait_ns"] / max(sends, 1) / 1e3}


def epoch_direct(rank, R):
    """The epoch engine (delivery "direct": route -> all-to-all -> dispatch ->
    all-to-all -> complete, wire v3 with the exact-size exchange) across processes."""
    n, M = 16384, 100_000
    tab, _ = table(n, R)
    st = torch.zeros(n // R + 1, dtype=torch.int64, device=DEV)
    ex = ActorExchange(tab, M, chunks=2, state=st, delivery="direct", comm="ipc")
    for k in range(4):
        req = B.gen_requests(M - 333 * rank, n, METHOD_CALC_MULTIPLY, seed=70 + 5 * rank + k, device=DEV)
        v, sts = ex.send_all(req)
        torch.cuda.synchronize()
        assert bool((sts == STATUS_OK).all()) and torch.equal(v, req.a0 * req.a1), k
    w = ex.last_wire
    assert w["S"] and w.get("engine", "epoch") != "sorted" and w["exact"], w
    return {"exact": bool(w["exact"]), "S": int(w["S"])}


def kill(rank, R):
    """The last rank SIGKILLs itself after two Sends.  The survivors' collectives
    wait for it only until the comm's timeout, then the next Send raises an
    IpcComm error that the elastic path classifies as a peer failure."""
    from ptype_amd.parallel.elastic import is_rank_failure

    n, M = 8192, 50_000
    tab, _ = table(n, R)
    st = torch.zeros(n // R + 1, dtype=torch.int64, device=DEV)
    ex = ActorExchange(tab, M, chunks=1, state=st, delivery="mailbox", mailbox_ordered=False, comm="ipc",
                       comm_timeout_s=3.0)
    for k in range(2):
        req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=k + 10 * rank, device=DEV)
        v, sts = ex.send(req)
        torch.cuda.synchronize()
        assert bool((sts == STATUS_OK).all())
    dist.barrier()
    if rank == R - 1:
        os.kill(os.getpid(), signal.SIGKILL)
    t0 = time.time()
    req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=99, device=DEV)
    v, sts = ex.send(req)  # enqueues; its waits end at the timeout on the device
    torch.cuda.synchronize()
    waited = time.time() - t0
    assert ex.ipc.failed, "the dead peer's collective was not detected"
    # no false successes: every message of the failed Send answers NotDelivered
    # (the completion reads the comm's failure word in stream order)
    counts = {int(k): int(c) for k, c in zip(*torch.unique(sts.cpu(), return_counts=True))}
    assert STATUS_OK not in counts and counts.get(STATUS_NOT_DELIVERED, 0) >= M * 0.99, counts
    try:
        ex.send(req)
    except RuntimeError as e:
        assert "IpcComm: peer" in str(e) and is_rank_failure(e), str(e)
        return {"raised": str(e)[:120], "waited_s": round(waited, 2), "statuses": counts}
    raise AssertionError("the Send after a peer's death did not raise")


if __name__ == "__main__":
    scenario, rank, world, port = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    torch.cuda.set_device(DEV)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    res = globals()[scenario](rank, world)
    if rank == 0:
        print("RESULT " + json.dumps(res), flush=True)
    sys.stdout.flush()
    os._exit(0)  # (no collective teardown: a peer may be gone)

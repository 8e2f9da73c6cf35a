"""The native epoch engine at R = 2..8 ranks on ONE GPU (csrc/hip/engine.hpp
FakeComm): R in-process ranks, each with its own host thread, stream, registry
mirror, actor state and batch, run the real multi-rank Send pipeline -- v3
agreement + packed slots, or v2 slots -- with the all-to-alls done as
event-ordered device copies.  Every reply is checked against its handler's
definition (no reference pipeline involved), and the actor state against the
messages that reached it.  Only RCCL's xGMI transport is not exercised here
(that is tests/test_engine_gpu.py's and test_packed_wire.py's world-1 RCCL run).
"""
import threading

import pytest
import torch

from ptype_amd.ops import batch as B
from ptype_amd.ops import hip
from ptype_amd.ops.records import (METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD, METHOD_ECHO, STATUS_NO_ACTOR,
                                   STATUS_OK)
from ptype_amd.ops.table import RegistryTable, actor_keys


def _rank_batch(r, M, n, mixed, big):
    g = torch.Generator().manual_seed(1000 + r)
    actor = torch.randint(0, n + 64, (M,), generator=g).to(torch.int32)  # ids >= n are unknown
    lim = 2**40 if big else 30000
    a0 = torch.randint(-lim, lim, (M,), generator=g)
    a1 = torch.randint(-lim, lim, (M,), generator=g)
    if mixed:
        m = torch.tensor([METHOD_CALC_MULTIPLY, METHOD_ECHO, METHOD_COUNTER_ADD])[torch.randint(0, 3, (M,), generator=g)]
        a0 = torch.where(m == METHOD_COUNTER_ADD, torch.ones_like(a0), a0)
    else:
        m = torch.full((M,), METHOD_CALC_MULTIPLY)
    return actor, a0, a1, m


@pytest.mark.gpu
@pytest.mark.parametrize("R,packed,chunks,mixed,big", [
    (2, True, 3, False, False), (4, True, 4, True, False), (8, True, 4, False, False),
    (8, True, 2, True, True), (3, False, 1, True, False), (8, False, 4, False, False)])
def test_gpu_engine_multirank(R, packed, chunks, mixed, big):
    from ptype_amd.parallel.exchange import ActorExchange

    n = 4000
    sizes = [60_000 + 7_777 * r for r in range(R)]
    Mmax = max(sizes)
    fc = hip().FakeComm(R)
    batches = [_rank_batch(r, sizes[r], n, mixed, big) for r in range(R)]
    results, errors = [None] * R, []
    states = [None] * R
    wires = [None] * R
    start = threading.Barrier(R)

    def run(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                tab = RegistryTable(2 * n, device="cuda")
                ids = torch.arange(n)
                tab.upsert(actor_keys(ids), (ids % R).to(torch.int32), (ids // R).to(torch.int32))
                tab.enable_directory(n, affine_world=R)
                st = torch.zeros(n // R + 1, dtype=torch.int64, device="cuda")
                # (delivery "direct": the epoch engine; "auto" at N > 1 is the sorted exchange now)
                ex = ActorExchange(tab, Mmax, chunks=chunks, state=st, packed=packed, fake=(fc, r), delivery="direct")
                actor, a0, a1, m = batches[r]
                req = B.MsgBatch(actor.cuda(), a0.cuda(), a1.cuda(), None,
                                 m.to(torch.int16).cuda() if mixed else METHOD_CALC_MULTIPLY)
                start.wait()
                val, sts = ex.send(req)
                s.synchronize()
                results[r] = (val.cpu(), sts.cpu())
                states[r] = st.cpu()
                wires[r] = ex.last_wire
        except BaseException as e:  # noqa: BLE001 - surfaced below
            errors.append((r, repr(e)))

    threads = [threading.Thread(target=run, args=(r,)) for r in range(R)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in threads), "a rank hung"
    assert not errors, errors
    counts = torch.zeros(n, dtype=torch.int64)
    for r in range(R):
        actor, a0, a1, m = batches[r]
        val, sts = results[r]
        known = actor.to(torch.int64) < n
        assert torch.equal(sts[~known], torch.full_like(sts[~known], STATUS_NO_ACTOR)), r
        assert bool((sts[known] == STATUS_OK).all()), (r, int((sts[known] != STATUS_OK).sum()))
        mul, echo = known & (m == METHOD_CALC_MULTIPLY), known & (m == METHOD_ECHO)
        assert torch.equal(val[mul], a0[mul] * a1[mul]), r
        assert torch.equal(val[echo], a0[echo]), r
        assert bool((val[~known] == 0).all())
        ca = known & (m == METHOD_COUNTER_ADD)
        counts += torch.bincount(actor[ca].to(torch.int64), minlength=n + 64)[:n]
        assert bool((val[ca] >= 1).all())
    # actor a lives on rank a % R in mailbox a // R: every CounterAdd arrived exactly once
    for r in range(R):
        mine = counts[r::R]
        assert torch.equal(states[r][: mine.numel()], mine), r
    if packed:
        L = wires[0]
        assert all(w["S"] == L["S"] and w["vb"] == L["vb"] for w in wires), "ranks disagree on the layout"
        if not mixed and not big:
            assert L["S"] == 2 and L["vb"] == 4, L  # 8-B requests, 4-B replies


@pytest.mark.gpu
@pytest.mark.parametrize("R,chunks,sync,link", [(8, 2, "values", 0.0), (8, 4, "events", 0.0), (4, 2, "values", 400.0),
                                                (2, 1, "values", 0.0)])
def test_gpu_engine_loopback(R, chunks, sync, link, monkeypatch):
    """FakeComm loopback (the bench's --loopback profiling mode): one rank runs an
    R-rank step with recv = send; every reply must still be its handler's value,
    with either cross-stream hand-off form and with the modelled link delay."""
    from ptype_amd.parallel.exchange import ActorExchange

    monkeypatch.setenv("PTYPE_TUNE", "stream_sync=" + ("1" if sync == "values" else "0"))
    n, M = 4096 * R, 300_000
    tab = RegistryTable(2 * n, device="cuda")
    ids = torch.arange(n)
    tab.upsert(actor_keys(ids), (ids % R).to(torch.int32), (ids // R).to(torch.int32))
    tab.enable_directory(n, affine_world=R)
    ex = ActorExchange(tab, M, chunks=chunks, state=torch.zeros(n // R, dtype=torch.int64, device="cuda"),
                       fake=(hip().FakeComm(R, loopback=True, link_gbps=link), 0), delivery="direct")
    for seed in (3, 4):
        req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=seed, device="cuda")
        val, st = ex.send(req)
        torch.cuda.synchronize()
        assert bool((st == STATUS_OK).all()) and torch.equal(val, req.a0 * req.a1)
    assert ex.last_wire["S"] == 2
    assert ex._engine.stream_values == (sync == "values")


@pytest.mark.gpu
@pytest.mark.parametrize("adaptive", [True, False])
def test_gpu_engine_zipf_skew_no_resend(adaptive, monkeypatch):
    """Zipf(1.1) traffic on the R = 8 pipeline.  With adaptive capacity the agreed
    slot size covers the busiest bucket: every message is delivered in ONE pass
    (no overflow, no host re-send round); the static capacity (mean + 8 sigma)
    overflows and needs send_all's rounds."""
    from ptype_amd.parallel.exchange import ActorExchange

    monkeypatch.setenv("PTYPE_TUNE", "adaptive_c=" + ("1" if adaptive else "0"))
    R, n, M = 8, 1 << 15, 200_000
    fc = hip().FakeComm(R)
    out, errors = [None] * R, []
    start = threading.Barrier(R)

    def run(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                tab = RegistryTable(2 * n, device="cuda")
                ids = torch.arange(n)
                tab.upsert(actor_keys(ids), (ids % R).to(torch.int32), (ids // R).to(torch.int32))
                tab.enable_directory(n, affine_world=R)
                st = torch.zeros(n // R, dtype=torch.int64, device="cuda")
                ex = ActorExchange(tab, M, chunks=2, state=st, fake=(fc, r), delivery="direct")
                req = B.gen_zipf_requests(M, n, 1.1, seed=10 + r, device="cuda")
                start.wait()
                v, sts = ex.send(req)  # one pass, no host re-send loop
                s.synchronize()
                over = int((sts == 4).sum())
                ok = bool(torch.equal(v[sts == STATUS_OK], (req.a0 * req.a1)[sts == STATUS_OK]))
                out[r] = (over, ok, ex.last_wire["C"], ex.last_wire["C_alloc"], ex.C)
        except BaseException as e:  # noqa: BLE001
            errors.append((r, repr(e)))

    threads = [threading.Thread(target=run, args=(r,)) for r in range(R)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not errors, errors
    Cs = {o[2] for o in out}
    assert len(Cs) == 1  # every rank agreed on one capacity
    for over, ok, C, C_alloc, C_static in out:
        assert ok
        if adaptive:
            assert over == 0 and C > C_static  # the hot bucket needed more than mean + 8 sigma
        else:
            assert C == C_static
    if not adaptive:
        assert sum(o[0] for o in out) > 0  # static slots overflow under this skew


@pytest.mark.gpu
@pytest.mark.parametrize("packed", [True, False])
def test_gpu_multirank_tells(packed):
    """Device tells across R = 4 in-process ranks: a token ring whose every hop is
    a ``Forward`` emitted by a dispatch kernel into the (LDS-staged) outbox and
    routed by the next epoch's exchange; every actor counts exactly the visits a
    plain simulation predicts."""
    from ptype_amd.ops.outbox import DeviceOutbox
    from ptype_amd.ops.records import METHOD_FORWARD
    from ptype_amd.parallel.exchange import ActorExchange

    R, n_per, T, hops, stride = 4, 5000, 3000, 9, 7
    n = n_per * R
    fc = hip().FakeComm(R)
    starts = [[(r * 1009 + 13 * t) % n for t in range(T)] for r in range(R)]
    states, errors, epochs = [None] * R, [], [None] * R
    start = threading.Barrier(R)

    def run(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                tab = RegistryTable(4 * n, device="cuda")
                ids = torch.arange(n)
                tab.upsert(actor_keys(ids), (ids % R).to(torch.int32), (ids // R).to(torch.int32))
                st = torch.zeros(n_per, dtype=torch.int64, device="cuda")
                ex = ActorExchange(tab, 2 * T, chunks=2, state=st, packed=packed, fake=(fc, r))
                ob = DeviceOutbox(2 * T, device="cuda")
                s0 = torch.tensor(starts[r], dtype=torch.int64)
                init = B.MsgBatch(s0.to(torch.int32).cuda(), ((s0 + stride) % n).cuda(),
                                  torch.full((T,), hops, dtype=torch.int64, device="cuda"),
                                  torch.full((T,), stride | (n << 32), dtype=torch.int64, device="cuda"),
                                  METHOD_FORWARD)
                start.wait()
                epochs[r], _ = ex.pump(ob, initial=init)
                s.synchronize()
                states[r] = st.cpu()
                assert ob.dropped == 0
        except BaseException as e:  # noqa: BLE001 - surfaced below
            errors.append((r, repr(e)))

    threads = [threading.Thread(target=run, args=(r,)) for r in range(R)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not errors, errors
    exp = torch.zeros(n, dtype=torch.int64)
    for ss in starts:
        for a in ss:
            for _ in range(hops + 1):
                exp[a] += 1
                a = (a + stride) % n
    for r in range(R):
        assert torch.equal(states[r], exp[r::R]), r  # actor a -> rank a % R, mailbox a // R
    assert all(e == hops for e in epochs), epochs


@pytest.mark.gpu
def test_gpu_replicated_prime_over_fakecomm_r4():
    """Prime served by 2 replica ranks (1, 3) of an R = 4 FakeComm
    pipeline; every rank's calls split over them exactly as its balancer's
    round robin picks (the replica_route kernel), Prime.Check answers right;
    after replica 1 is lost every call lands on rank 3."""
    from ptype_amd.parallel.exchange import ActorExchange
    from ptype_amd.parallel.replicas import ReplicaRouter
    from ptype_amd.ops.records import METHOD_PRIME_CHECK

    R, P = 4, 512
    n = P * R
    fc = hip().FakeComm(R)
    recs = [{"rank": r, "world": R, "count": P, "node": f"p{r}", "replica": True, "address": f"10.0.0.{r}",
             "port": 7000} for r in (1, 3)]
    sizes = [20_000 + 999 * r for r in range(R)]
    states, results, errors = [None] * R, [None] * R, []
    start = threading.Barrier(R)

    def run(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                tab = RegistryTable(2 * n, device="cuda")
                ids = torch.arange(n)
                tab.upsert(actor_keys(ids), (ids % R).to(torch.int32), (ids // R).to(torch.int32))
                tab.enable_directory(n, affine_world=R)
                st = torch.zeros(P, dtype=torch.int64, device="cuda")
                ex = ActorExchange(tab, max(sizes), chunks=2, state=st, fake=(fc, r))
                router = ReplicaRouter("Prime", R, f"10.1.0.{r}", 3, records=recs)
                M = sizes[r]
                a = (torch.arange(M, device="cuda") % P).to(torch.int32)
                start.wait()
                # (send_all, as Client.Send: the sorted exchange's first Sends run at the start-up
                # capacity, and all of this traffic lands on the two replicas -- overflow, re-sent)
                _, s1 = ex.send_all(B.MsgBatch(router.route(a), torch.ones(M, dtype=torch.int64, device="cuda"), None,
                                               None, METHOD_COUNTER_ADD))
                t = torch.tensor([97, 91, 62, 273, 7919], dtype=torch.int64, device="cuda")
                pv, ps = ex.send_all(B.MsgBatch(router.route(torch.arange(5, dtype=torch.int32, device="cuda")),
                                                torch.full_like(t, 2), t, t, METHOD_PRIME_CHECK))
                s.synchronize()
                start.wait()
                c1 = st.clone()
                router.set_records(recs[1:])  # replica 1 lost
                _, s2 = ex.send_all(B.MsgBatch(router.route(a), torch.ones(M, dtype=torch.int64, device="cuda"), None,
                                               None, METHOD_COUNTER_ADD))
                s.synchronize()
                results[r] = (s1.cpu(), ps.cpu(), pv.cpu(), s2.cpu())
                states[r] = (c1.cpu(), (st - c1).cpu())
        except BaseException as e:  # noqa: BLE001
            errors.append((r, repr(e)))

    threads = [threading.Thread(target=run, args=(r,)) for r in range(R)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in threads), "a rank hung"
    assert not errors, errors
    want1 = {q: torch.zeros(P, dtype=torch.int64) for q in (1, 3)}
    for r in range(R):
        s1, ps, pv, s2 = results[r]
        assert bool((s1 == STATUS_OK).all()) and bool((s2 == STATUS_OK).all()) and bool((ps == STATUS_OK).all())
        assert pv.tolist() == [97, 7, 2, 3, 7919]
        for i in range(sizes[r]):
            want1[(1, 3)[(1 + i) % 2]][i % P] += 1
    total = sum(torch.bincount(torch.arange(sizes[r]) % P, minlength=P) for r in range(R))
    for r in range(R):
        c1, c2 = states[r]
        if r in (1, 3):
            assert torch.equal(c1, want1[r]), r
            assert torch.equal(c2, total if r == 3 else torch.zeros(P, dtype=torch.int64)), r
        else:
            assert int(c1.sum()) == 0 and int(c2.sum()) == 0


@pytest.mark.gpu
def test_gpu_multirank_device_pump_no_host_round_trip_per_epoch(monkeypatch):
    """the FakeComm R = 4 token ring on the device-counted
    multi-rank pump -- each epoch routes its outbox bank by the bank's DEVICE
    count (idle slots sealed), and the ranks agree on what is left with a device
    all-reduce once per group of epochs: no host agreement per epoch (counted),
    and every actor's visits match a plain simulation."""
    from ptype_amd.ops.outbox import DeviceOutbox
    from ptype_amd.ops.records import METHOD_FORWARD
    from ptype_amd.parallel.exchange import ActorExchange

    R, n_per, T, hops, stride = 4, 3000, 1500, 11, 5
    n = n_per * R
    cap = 3 * T
    fc = hip().FakeComm(R)
    starts = [[(r * 701 + 17 * t) % n for t in range(T)] for r in range(R)]
    states, errors, epochs, agrees, sealed = [None] * R, [], [None] * R, [0] * R, [0] * R
    orig = ActorExchange._agree_max

    def counting(self, v):
        agrees[self.rank] += 1
        return orig(self, v)

    monkeypatch.setattr(ActorExchange, "_agree_max", counting)
    start = threading.Barrier(R)

    def run(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                tab = RegistryTable(4 * n, device="cuda")
                ids = torch.arange(n)
                tab.upsert(actor_keys(ids), (ids % R).to(torch.int32), (ids // R).to(torch.int32))
                st = torch.zeros(n_per, dtype=torch.int64, device="cuda")
                ex = ActorExchange(tab, cap, chunks=1, state=st, slack=3.0, fake=(fc, r))
                ob = DeviceOutbox(cap, device="cuda")
                assert ex._device_pump_multi_ok(ob)
                s0 = torch.tensor(starts[r], dtype=torch.int64)
                init = B.MsgBatch(s0.to(torch.int32).cuda(), ((s0 + stride) % n).cuda(),
                                  torch.full((T,), hops, dtype=torch.int64, device="cuda"),
                                  torch.full((T,), stride | (n << 32), dtype=torch.int64, device="cuda"),
                                  METHOD_FORWARD)
                start.wait()
                epochs[r], _ = ex.pump(ob, initial=init, check_every=4)
                s.synchronize()
                states[r] = st.cpu()
                sealed[r] = ex.stats().pump_sealed
                assert ob.dropped == 0
        except BaseException as e:  # noqa: BLE001 - surfaced below
            errors.append((r, repr(e)))

    threads = [threading.Thread(target=run, args=(r,)) for r in range(R)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in threads), "a rank hung"
    assert not errors, errors
    exp = torch.zeros(n, dtype=torch.int64)
    for ss in starts:
        for a in ss:
            for _ in range(hops + 1):
                exp[a] += 1
                a = (a + stride) % n
    for r in range(R):
        assert torch.equal(states[r], exp[r::R]), r
    assert all(e == hops for e in epochs), epochs
    assert agrees == [1] * R, agrees  # the initial batch's size only: none per epoch
    assert all(x > 0 for x in sealed), sealed  # the device-counted path ran

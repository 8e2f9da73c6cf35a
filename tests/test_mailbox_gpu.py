"""HBM actor mailboxes (K2 enqueue / K3 drain / persistent consumer) on MI355X.

Numerics: stateless replies are compared exactly with the plain-PyTorch handler
reference; ordered (SeqFold) traffic is audited by chain reconstruction
(ops.mailbox.audit_fold): every actor's replies must chain its state from
before to after the Send through every message exactly once, which also
exposes the order each actor ran its messages in (FIFO checks).
"""
import os
import subprocess
import sys
import textwrap

import pytest
import torch

from ptype_amd.ops import batch as B
from ptype_amd.ops.mailbox import Mailboxes, audit_fold
from ptype_amd.ops.records import (METHOD_CALC_MULTIPLY, METHOD_PRIME_CHECK, METHOD_SEQ_FOLD, STATUS_NO_ACTOR,
                                   STATUS_OK, STATUS_OVERFLOW)
from ptype_amd.ops.table import RegistryTable, actor_keys
from ptype_amd.parallel.exchange import ActorExchange

from conftest import ROOT

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def placed_table(n, seed=7, directory=True):
    """Every actor on rank 0 at a random mailbox (a permutation): routes must read the mirror."""
    t = RegistryTable(2 * n, device=DEV)
    ids = torch.arange(n)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(seed))
    t.upsert(actor_keys(ids), torch.zeros(n, dtype=torch.int32), perm.to(torch.int32))
    if directory:
        t.enable_directory(n)
    return t, perm


def fold_batch(M, n_actors, seed):
    g = torch.Generator().manual_seed(seed)
    actor = torch.randint(0, n_actors, (M,), generator=g, dtype=torch.int32)
    a0 = torch.randint(-(1 << 40), 1 << 40, (M,), generator=g, dtype=torch.int64)
    return B.MsgBatch(actor.to(DEV), a0.to(DEV), None, None, METHOD_SEQ_FOLD)


@pytest.mark.parametrize("directory", [True, False])
def test_mailbox_send_calculator_matches_reference(directory):
    n, M = 1 << 15, 1 << 20
    t, _ = placed_table(n, directory=directory)
    mb = Mailboxes(DEV, shards=256, slots=1 << 14)
    req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=3, device=DEV)
    val, st = mb.send(req, t, None)
    torch.cuda.synchronize()
    assert bool((st == STATUS_OK).all())
    assert torch.equal(val, req.a0 * req.a1)
    s = mb.stats()
    # (a message whose fields outgrow the first Send's 8-B record widths spills: run from the batch)
    assert s["enqueued"] + s["spilled"] == M and s["processed"] == M and s["overflow"] == 0 and s["holes"] == 0
    ctr = mb.shard_counters()
    assert (ctr[:, 0] == ctr[:, 2]).all() and int(ctr[:, 0].sum()) == M  # every ring drained


@pytest.mark.parametrize("M", [1 << 20, 5 << 20])
def test_mailbox_stateless_rank_byte_route(M):
    """A stateless uniform Send on the directory resolves ranks only (route mode 3,
    the rank byte table; mode 4, its 2-bit presence map staged in LDS, for the
    one-pass sort) and its records carry actor ids: exact replies for
    directory ids, ids past the directory (hash probe) and unregistered ids on both
    sides of its end -- through the fused Send (1 Mi) and the two-kernel one with
    8-B records (5 Mi)."""
    n = 1 << 15
    t = RegistryTable(4 * n, device=DEV)
    ids = torch.cat([torch.arange(n), torch.arange(n + 100, n + 1100)])
    perm = torch.randperm(ids.numel(), generator=torch.Generator().manual_seed(11))
    t.upsert(actor_keys(ids), torch.zeros(ids.numel(), dtype=torch.int32), perm.to(torch.int32))
    t.enable_directory(n + 50)  # ids n..n+49: in the directory, unregistered
    g = torch.Generator().manual_seed(12)
    actor = torch.randint(0, n + 3000, (M,), generator=g, dtype=torch.int32)
    a0 = torch.randint(-(1 << 15), 1 << 15, (M,), generator=g, dtype=torch.int64)
    a1 = torch.randint(-(1 << 15), 1 << 15, (M,), generator=g, dtype=torch.int64)
    req = B.MsgBatch(actor.to(DEV), a0.to(DEV), a1.to(DEV), None, METHOD_CALC_MULTIPLY)
    mb = Mailboxes(DEV, shards=256, slots=1 << 16)
    for _ in range(2):  # (the second Send runs on the widths the first one measured)
        val, st = mb.send(req, t, None, ordered=False)
        torch.cuda.synchronize()
        # the fused Send gathers rank bytes (3); the one-pass sort stages the directory's
        # presence map in LDS (4)
        assert mb.last_route == (3 if M <= 2 << 20 else 4)
        a = actor.to(DEV)
        known = (a < n) | ((a >= n + 100) & (a < n + 1100))
        assert torch.equal(st, torch.where(known, STATUS_OK, STATUS_NO_ACTOR).to(torch.int32))
        assert torch.equal(val[known], (req.a0 * req.a1)[known])
    ctr = mb.shard_counters()
    assert (ctr[:, 0] == ctr[:, 2]).all()  # every ring drained


@pytest.mark.parametrize("sharding", ["actor", "arrival"])
def test_mailbox_unknown_actor_and_three_args(sharding):
    n, M = 4096, 50_000
    t, _ = placed_table(n)
    mb = Mailboxes(DEV, shards=64, slots=4096)
    g = torch.Generator().manual_seed(5)
    actor = torch.randint(0, n + 500, (M,), generator=g, dtype=torch.int32)  # ids >= n are unregistered
    lo = torch.randint(0, 50, (M,), generator=g)
    req = B.MsgBatch(actor.to(DEV), lo.to(DEV), (lo + 10).to(DEV), torch.randint(2, 5000, (M,), generator=g).to(DEV),
                     METHOD_PRIME_CHECK)
    val, st = mb.send(req, t, None, sharding=sharding)
    torch.cuda.synchronize()
    ref_v, ref_s = B._handler_ref(torch.full((M,), METHOD_PRIME_CHECK), actor.long(), lo, lo + 10,
                                  req.a2.cpu(), None)
    known = actor < n
    assert torch.equal(st.cpu()[~known], torch.full((int((~known).sum()),), STATUS_NO_ACTOR, dtype=torch.int32))
    assert bool((st.cpu()[known] == STATUS_OK).all())
    assert torch.equal(val.cpu()[known], ref_v[known])


def test_mailbox_seqfold_exactly_once_and_fifo_1m():
    """1 M ordered messages to 4096 actors in two Sends: every actor's replies chain
    exactly once, and all of Send 1 ran before any of Send 2 (FIFO across Sends)."""
    n, M = 4096, 1 << 19
    t, perm = placed_table(n)
    state = torch.randint(0, 1 << 30, (n,), dtype=torch.int64, device=DEV)
    ex = ActorExchange(t, M, state=state)  # auto delivery: a uniform ordered method -> mailboxes
    s0 = state.cpu().clone()
    r1 = fold_batch(M, n, 11)
    v1, st1 = ex.send(r1)
    torch.cuda.synchronize()
    s1 = state.cpu().clone()
    r2 = fold_batch(M, n, 12)
    v2, st2 = ex.send(r2)
    torch.cuda.synchronize()
    s2 = state.cpu().clone()
    assert ex.mailboxes is not None
    mbox1, mbox2 = perm[r1.actor.cpu().long()], perm[r2.actor.cpu().long()]
    ok, info = audit_fold(mbox1, r1.a0.cpu(), v1.cpu(), st1.cpu(), s0, s1)
    assert ok, info
    ok, info = audit_fold(mbox2, r2.a0.cpu(), v2.cpu(), st2.cpu(), s1, s2)
    assert ok, info
    # both Sends together also chain: Send 2 continued exactly where Send 1 left every actor
    ok, info = audit_fold(torch.cat([mbox1, mbox2]), torch.cat([r1.a0.cpu(), r2.a0.cpu()]),
                          torch.cat([v1.cpu(), v2.cpu()]), torch.cat([st1.cpu(), st2.cpu()]), s0, s2)
    assert ok, info
    order = info
    x = next(iter(order))
    assert all(i < M for i in order[x][: int((mbox1 == x).sum())])  # Send 1's messages first
    st = ex.stats()
    assert st.mailbox["processed"] == 2 * M and st.mailbox["serialised"] > 0  # same-actor windows ran serialised


def test_mailbox_overflow_is_answered_and_resent():
    """Rings too small for the batch: the excess is answered STATUS_OVERFLOW at enqueue,
    never half-applied; send_all re-sends it until everything ran exactly once."""
    n, M = 256, 20_000
    t, perm = placed_table(n)
    state = torch.zeros(n, dtype=torch.int64, device=DEV)
    ex = ActorExchange(t, M, state=state, delivery="mailbox", mailbox_shards=4, mailbox_slots=1024)
    req = fold_batch(M, n, 21)
    v, st = ex.send(req)
    torch.cuda.synchronize()
    first = st.cpu()
    assert int((first == STATUS_OVERFLOW).sum()) > 0 and int((first == STATUS_OK).sum()) > 0
    state.zero_()
    ex.mailboxes.reset()
    v, st = ex.send_all(req, max_epochs=64)
    torch.cuda.synchronize()
    ok, info = audit_fold(perm[req.actor.cpu().long()], req.a0.cpu(), v.cpu(), st.cpu(), torch.zeros(n, dtype=torch.long),
                          state.cpu())
    assert ok, info
    assert ex.counters.resends > 0


@pytest.mark.parametrize("shards,slots,blocks", [(128, 1 << 12, 8), (256, 1 << 10, 16), (64, 1 << 13, 4)])
def test_mailbox_persistent_consumer_live_enqueue(shards, slots, blocks):
    """The persistent consumer drains while batches keep arriving from another stream;
    after stop() every message ran exactly once, batches in submission order.  Rings
    smaller than the traffic: slots are recycled while the consumer runs."""
    n, M, batches = 2048, 1 << 16, 6
    t, perm = placed_table(n)
    state = torch.randint(0, 1 << 20, (n,), dtype=torch.int64, device=DEV)
    s0 = state.cpu().clone()
    mb = Mailboxes(DEV, shards=shards, slots=slots)
    out_v = torch.full((M * batches,), -1, dtype=torch.int64, device=DEV)
    out_s = torch.full((M * batches,), -1, dtype=torch.int32, device=DEV)
    reqs = [fold_batch(M, n, 100 + b) for b in range(batches)]
    torch.cuda.synchronize()
    mb.start(state, out_v, out_s, blocks=blocks, max_s=20.0)
    prod = torch.cuda.Stream(DEV)
    with torch.cuda.stream(prod):
        for b, r in enumerate(reqs):
            mb.enqueue(r, t, out_v, out_s, origin_base=b * M, live=True)
    prod.synchronize()
    mb.stop()
    torch.cuda.synchronize()
    st = out_s.cpu()
    # a full ring answers STATUS_OVERFLOW instead of waiting: those messages never ran
    ran = st == STATUS_OK
    assert bool(((st == STATUS_OK) | (st == STATUS_OVERFLOW)).all())
    assert int(ran.sum()) > M  # the consumer kept up with most of it
    actor = torch.cat([r.actor.cpu() for r in reqs]).long()
    a0 = torch.cat([r.a0.cpu() for r in reqs])
    ok, info = audit_fold(perm[actor[ran]], a0[ran], out_v.cpu()[ran], st[ran], s0, state.cpu())
    assert ok, info
    s = mb.stats()
    assert s["processed"] == int(ran.sum()) and s["consumer_processed"] == int(ran.sum())
    # FIFO across batches: per actor, messages ran in batch order
    idx = torch.nonzero(ran).flatten()
    for x, seq in list(info.items())[:64]:
        b = [int(idx[i]) // M for i in seq]
        assert b == sorted(b)


def test_mailbox_send_graph_replay():
    n, M = 1 << 14, 1 << 18
    t, _ = placed_table(n)
    state = torch.zeros(n, dtype=torch.int64, device=DEV)
    ex = ActorExchange(t, M, state=state, delivery="mailbox")
    req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=1, device=DEV)
    val = torch.empty(M, dtype=torch.int64, device=DEV)
    st = torch.empty(M, dtype=torch.int32, device=DEV)
    g = ex.capture(req, val, st)
    for s in range(3):
        B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=40 + s, device=DEV, out=req)
        g.replay()
        torch.cuda.synchronize()
        assert bool((st == STATUS_OK).all()) and torch.equal(val, req.a0 * req.a1)


@pytest.mark.parametrize("R,ordered,packed", [(4, True, True), (3, False, True), (4, True, False), (3, False, False)])
def test_mailbox_delivery_on_receipt_multirank(R, ordered, packed, monkeypatch):
    """N > 1: every rank's received records go through its HBM mailboxes (K2 on
    receipt from the request regions, K3 into the reply regions), on the engine's
    real multi-rank pipeline (FakeComm ranks, one GPU).  Ordered: SeqFold traffic
    from every rank to every rank's actors, audited per actor across all senders
    (exactly once, serialised).  Unordered: calculator replies exact.  ``packed``:
    wire v3 records are enqueued straight from the packed regions and the drain's
    replies are packed into v3 reply regions; else wire v2."""
    import threading

    from ptype_amd.ops import hip

    # the epoch engine's delivery on receipt (the sorted exchange is tested in test_sorted_exchange_gpu.py)
    monkeypatch.setenv("PTYPE_TUNE", "sorted_exchange=0")
    n, M = 4096, 60_000
    fc = hip().FakeComm(R)
    res, errors = [None] * R, []
    start = threading.Barrier(R)
    states0 = [torch.randint(0, 1 << 30, (n // R + 1,), dtype=torch.int64, generator=torch.Generator().manual_seed(r))
               for r in range(R)]

    def run(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                tab = RegistryTable(2 * n, device="cuda")
                ids = torch.arange(n)
                tab.upsert(actor_keys(ids), (ids % R).to(torch.int32), (ids // R).to(torch.int32))
                tab.enable_directory(n, affine_world=R)
                st = states0[r].to("cuda")
                ex = ActorExchange(tab, M, chunks=2, state=st, fake=(fc, r), delivery="mailbox",
                                   mailbox_ordered=ordered, mailbox_shards=64, packed=packed)
                req = fold_batch(M, n, 300 + r) if ordered else B.gen_requests(M, n, METHOD_CALC_MULTIPLY,
                                                                                 seed=300 + r, device="cuda")
                start.wait()
                v, sts = ex.send(req)
                s.synchronize()
                assert (ex.last_wire["S"] > 0) == packed, ex.last_wire
                res[r] = (req.actor.cpu().long(), req.a0.cpu(), None if ordered else req.a1.cpu(), v.cpu(), sts.cpu(),
                          st.cpu(), ex.stats().mailbox)
        except BaseException as e:  # noqa: BLE001
            errors.append((r, repr(e)))

    ths = [threading.Thread(target=run, args=(r,)) for r in range(R)]
    [t.start() for t in ths]
    [t.join(timeout=240) for t in ths]
    assert not errors, errors
    for r in range(R):
        assert res[r][6]["processed"] > 0 and res[r][6]["enqueued"] == res[r][6]["processed"]
    if not ordered:
        for actor, a0, a1, v, sts, _, _ in res:
            assert bool((sts == STATUS_OK).all()) and torch.equal(v, a0 * a1)
        return
    actor = torch.cat([x[0] for x in res])
    a0 = torch.cat([x[1] for x in res])
    v = torch.cat([x[3] for x in res])
    sts = torch.cat([x[4] for x in res])
    # global mailbox key: owner rank * (n // R + 1) + local mailbox
    P = n // R + 1
    key = (actor % R) * P + actor // R
    before = torch.cat(states0)
    after = torch.cat([x[5] for x in res])
    ok, info = audit_fold(key, a0, v, sts, before, after)
    assert ok, info


# ---------------------------------------------------------------- sorted epoch mailboxes
# (csrc/hip/mailbox_sort.hip: counting-sort enqueue into message-ordered rings,
# parallel / LDS-binned ordered drains)

@pytest.mark.parametrize("sharding", ["actor", "arrival"])
@pytest.mark.parametrize("M", [1, 5000, 1 << 20])
def test_sorted_mailbox_calculator_exact(sharding, M):
    n = 1 << 15
    t, _ = placed_table(n)
    mb = Mailboxes(DEV, shards=256, slots=1 << 14)
    for rep in range(2):  # the second Send starts where the first left every ring
        req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=3 + rep, device=DEV)
        val, st = mb.send(req, t, None, sharding=sharding)
        torch.cuda.synchronize()
        assert bool((st == STATUS_OK).all())
        assert torch.equal(val, req.a0 * req.a1)
    s = mb.stats()
    assert s["enqueued"] == 2 * M and s["processed"] == 2 * M and s["overflow"] == 0 and s["holes"] == 0
    ctr = mb.shard_counters()
    assert (ctr[:, 0] == ctr[:, 2]).all() and int(ctr[:, 0].sum()) == 2 * M


@pytest.mark.parametrize("sharding", ["actor", "arrival"])
def test_sorted_mailbox_partial_spill_then_clean_send(sharding):
    """Rings that hold only part of a Send: the early tiles / runs go through the
    rings, the rest spill (run from the batch by the drain: the ring-order drain
    takes a spilled tile in message order).  Every message is answered exactly,
    misses included, and the next Send finds every ring consumed."""
    n, M = 4096, 300_000
    t, _ = placed_table(n)
    mb = Mailboxes(DEV, shards=16, slots=8192)
    g = torch.Generator().manual_seed(11)
    for rep in range(2):
        actor = torch.randint(0, n + 300, (M,), generator=g, dtype=torch.int32)  # ids >= n: no actor
        a0 = torch.randint(-(1 << 31), 1 << 31, (M,), generator=g, dtype=torch.int64)
        a1 = torch.randint(-(1 << 20), 1 << 20, (M,), generator=g, dtype=torch.int64)
        req = B.MsgBatch(actor.to(DEV), a0.to(DEV), a1.to(DEV), None, METHOD_CALC_MULTIPLY)
        val, st = mb.send(req, t, None, sharding=sharding)
        torch.cuda.synchronize()
        known = actor < n
        st, val = st.cpu(), val.cpu()
        assert bool((st[known] == STATUS_OK).all()) and bool((st[~known] == STATUS_NO_ACTOR).all())
        assert torch.equal(val[known], (a0 * a1)[known])
        ctr = mb.shard_counters()
        assert (ctr[:, 0] == ctr[:, 2]).all()  # consumed: tail == head on every shard
    s = mb.stats()
    assert s["spilled"] > 0 and s["overflow"] == 0 and s["holes"] == 0
    assert s["processed"] == s["enqueued"] + s["spilled"], s


def test_sorted_vs_tagged_kernels_same_replies():
    n, M = 1 << 12, 200_000
    t, _ = placed_table(n)
    req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=8, device=DEV)
    outs = []
    for sort in (True, False):
        mb = Mailboxes(DEV, shards=64, slots=1 << 14)
        outs.append(mb.send(req, t, None, sort=sort))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("shards,n", [(256, 4096), (4, 32768)])  # (4, 32768): 8192 actors per shard, state in HBM
def test_sorted_mailbox_seqfold_fifo_within_a_send(shards, n):
    """Ordered drain: every actor's messages run one at a time in MESSAGE order
    (the rings are a stable sort of the batch), checked by chain reconstruction;
    64-bit arguments exercise the long record form."""
    M = 1 << 18
    t, perm = placed_table(n)
    state = torch.randint(0, 1 << 30, (n,), dtype=torch.int64, device=DEV)
    s0 = state.cpu().clone()
    mb = Mailboxes(DEV, shards=shards, slots=1 << 17)
    req = fold_batch(M, n, 41)
    v, st = mb.send(req, t, state)
    torch.cuda.synchronize()
    ok, order = audit_fold(perm[req.actor.cpu().long()], req.a0.cpu(), v.cpu(), st.cpu(), s0, state.cpu())
    assert ok, order
    for x, seq in order.items():
        assert seq == sorted(seq), f"actor {x} ran its messages out of message order"
    s = mb.stats()
    assert s["processed"] == M and s["serialised"] > 0 and s["holes"] == 0


def test_sorted_mailbox_mixed_methods_keep_actor_fifo():
    """A method column mixing SeqFold (ordered), Calculator.Multiply and Echo: the
    ordered drain runs all of an actor's messages in message order."""
    from ptype_amd.ops.records import METHOD_ECHO

    n, M = 2048, 300_000
    t, perm = placed_table(n)
    g = torch.Generator().manual_seed(77)
    actor = torch.randint(0, n, (M,), generator=g, dtype=torch.int32)
    meth = torch.tensor([METHOD_SEQ_FOLD, METHOD_CALC_MULTIPLY, METHOD_ECHO])[torch.randint(0, 3, (M,), generator=g)]
    a0 = torch.randint(-(1 << 20), 1 << 20, (M,), generator=g, dtype=torch.int64)
    a1 = torch.randint(-(1 << 20), 1 << 20, (M,), generator=g, dtype=torch.int64)
    req = B.MsgBatch(actor.to(DEV), a0.to(DEV), a1.to(DEV), None, meth.to(torch.int32).to(DEV))
    state = torch.randint(0, 1 << 30, (n,), dtype=torch.int64, device=DEV)
    s0 = state.cpu().clone()
    mb = Mailboxes(DEV, shards=128, slots=1 << 15)
    v, st = mb.send(req, t, state)
    torch.cuda.synchronize()
    v, st = v.cpu(), st.cpu()
    assert bool((st == STATUS_OK).all())
    mul, echo, fold = meth == METHOD_CALC_MULTIPLY, meth == METHOD_ECHO, meth == METHOD_SEQ_FOLD
    assert torch.equal(v[mul], (a0 * a1)[mul]) and torch.equal(v[echo], a0[echo])
    ok, order = audit_fold(perm[actor[fold].long()], a0[fold], v[fold], st[fold], s0, state.cpu())
    assert ok, order
    assert all(seq == sorted(seq) for seq in order.values())


def test_sorted_mailbox_overflow_keeps_fifo_prefix():
    """Rings smaller than an actor's traffic: the overflowed messages are each
    shard's LAST ones (the accepted prefix stays FIFO), answered STATUS_OVERFLOW."""
    n, M = 64, 20_000
    t, perm = placed_table(n)
    state = torch.zeros(n, dtype=torch.int64, device=DEV)
    mb = Mailboxes(DEV, shards=4, slots=1024)
    req = fold_batch(M, n, 9)
    v, st = mb.send(req, t, state)
    torch.cuda.synchronize()
    st = st.cpu()
    over = st == STATUS_OVERFLOW
    assert int(over.sum()) == M - 4 * 1024 and int((st == STATUS_OK).sum()) == 4 * 1024
    shard = perm[req.actor.cpu().long()] % 4
    for s in range(4):
        idx = torch.nonzero(shard == s).flatten()
        ok_s = ~over[idx]
        assert bool(ok_s[:1024].all()) and not bool(ok_s[1024:].any())  # the first 1024 in message order ran


def test_sorted_mailbox_stateless_spills_instead_of_overflow():
    """a stateless batch whose rings are far too small (all traffic
    on 4 x 1024 slots) spills: every message is answered by the drain straight
    from the batch -- no STATUS_OVERFLOW, so ``send_all`` needs no re-send round
    and no host read of an overflow count."""
    n, M = 64, 50_000
    t, _ = placed_table(n)
    mb = Mailboxes(DEV, shards=4, slots=1024)
    req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=5, device=DEV)
    v, st = mb.send(req, t, None)
    torch.cuda.synchronize()
    assert bool((st == STATUS_OK).all()) and torch.equal(v, req.a0 * req.a1)
    s = mb.stats()
    assert s["overflow"] == 0 and s["spilled"] == M - 4 * 1024 and s["processed"] == M, s
    # through the exchange: send_all takes the no-overflow exit (no re-send, no count read)
    ex = ActorExchange(t, M, chunks=1, delivery="mailbox", mailbox_shards=4, mailbox_slots=1024)
    calls = []
    orig = torch.Tensor.sum
    try:
        torch.Tensor.sum = lambda self, *a, **k: calls.append(1) or orig(self, *a, **k)
        v2, st2 = ex.send_all(req)
    finally:
        torch.Tensor.sum = orig
    torch.cuda.synchronize()
    assert torch.equal(v2, req.a0 * req.a1) and bool((st2 == STATUS_OK).all())
    assert ex.counters.resends == 0 and not calls


@pytest.mark.parametrize("fused", ["1", "0"])
def test_sorted_mailbox_8b_records_spill_what_does_not_fit(fused):
    """8-B ring records (stateless one-method batches): the mailbox field is
    sized from the state (1000 entries: 10 bits) and the arguments share the
    rest, so actors past mailbox 1023 and arguments of 40 bits cannot be
    encoded -- those messages spill (run straight from the batch) and every
    reply is still exact; the rest ride 8-B records.  Fused and separate
    kernels, in a subprocess (the switches are read once per process)."""
    code = textwrap.dedent('''
        import torch
        from ptype_amd.ops import batch as B
        from ptype_amd.ops.mailbox import Mailboxes
        from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, STATUS_OK
        from test_mailbox_gpu import placed_table
        n, M = 5000, 300_000
        t, _ = placed_table(n)
        state = torch.zeros(1000, dtype=torch.int64, device="cuda")
        mb = Mailboxes("cuda", shards=256, slots=16384)
        for k in range(3):
            req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=11 + k, device="cuda")
            if k == 1:
                req.a0[::97] = (1 << 40) + 3
                req.a1[::89] = -(1 << 38)
            v, st = mb.send(req, t, state, ordered=False)
            torch.cuda.synchronize()
            assert bool((st == STATUS_OK).all()), int((st != STATUS_OK).sum())
            assert torch.equal(v, req.a0 * req.a1), k
        s = mb.stats()
        assert s["overflow"] == 0 and s["spilled"] > 0 and s["processed"] == 3 * M, s
        print("OK", s["spilled"])
    ''')
    # (mbox_rec8=1: this batch size would take 16-B records by default)
    env = dict(os.environ, PTYPE_TUNE=f"mbox_fused={fused},mbox_rec8=1",
               PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "tests")]))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


@pytest.mark.parametrize("fused", ["1", "0"])
def test_sorted_mailbox_wide_pure_records_and_back_to_8b(fused):
    """Full-range int64 arguments of a stateless rank-routed batch: the Send that
    first meets them spills them (its 8-B widths were narrow), the next ones take
    the 18-B wide pure records (16 B {a0, a1} + the u16 place; no mailbox -- the
    methods read none), and once the values are narrow again the batches return to
    8-B records.  Every reply exact, unknown actors answered, no overflow."""
    code = textwrap.dedent('''
        import torch
        from ptype_amd.ops import batch as B
        from ptype_amd.ops.mailbox import Mailboxes
        from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, STATUS_NO_ACTOR, STATUS_OK
        from ptype_amd.ops.table import RegistryTable, actor_keys
        n, M = 1 << 14, 600_000
        t = RegistryTable(4 * n, device="cuda")
        ids = torch.arange(n)
        perm = torch.randperm(n, generator=torch.Generator().manual_seed(5))
        t.upsert(actor_keys(ids), torch.zeros(n, dtype=torch.int32), perm.to(torch.int32))
        t.enable_directory(n)
        mb = Mailboxes("cuda", shards=256, slots=16384)
        seen = []
        for k, wide in enumerate([False, True, True, True, False, False]):
            g = torch.Generator().manual_seed(40 + k)
            actor = torch.randint(0, n + 500, (M,), generator=g, dtype=torch.int32)
            lo, hi = (-(1 << 63), (1 << 63) - 1) if wide else (-(1 << 15), 1 << 15)
            a0 = torch.randint(lo, hi, (M,), generator=g, dtype=torch.int64)
            a1 = torch.randint(lo, hi, (M,), generator=g, dtype=torch.int64)
            req = B.MsgBatch(actor.cuda(), a0.cuda(), a1.cuda(), None, METHOD_CALC_MULTIPLY)
            v, st = mb.send(req, t, None, ordered=False)
            torch.cuda.synchronize()
            assert mb.last_route in (3, 4)
            known = req.actor < n
            assert torch.equal(st, torch.where(known, STATUS_OK, STATUS_NO_ACTOR).to(torch.int32)), k
            assert torch.equal(v[known], (req.a0 * req.a1)[known]), k
            seen.append(int(mb.last_record_bytes))
        s = mb.stats()
        assert s["overflow"] == 0 and s["holes"] == 0, s
        assert seen == [8, 8, 18, 18, 18, 8], seen
        print("OK", seen, s["spilled"])
    ''')
    # (mbox_rec8=1: this batch size would take 16-B records by default)
    env = dict(os.environ, PTYPE_TUNE=f"mbox_fused={fused},mbox_rec8=1",
               PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "tests")]))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


def test_live_mailbox_sustained_overload_keeps_consumer_rate():
    """two producer streams keep a persistent consumer ~3x over
    capacity for more than a second.  A full ring reserves nothing (no holes),
    so the consumer keeps draining at its unloaded rate; every STATUS_OK
    message ran exactly once (CounterAdd(1): each actor's OK replies are exactly
    1..k and its final state is k), everything else was answered OVERFLOW."""
    import time

    from ptype_amd.ops.records import METHOD_COUNTER_ADD

    n, S, Q = 4096, 256, 4096
    t, perm = placed_table(n)
    state = torch.zeros(n, dtype=torch.int64, device=DEV)
    mb = Mailboxes(DEV, shards=S, slots=Q)

    def consumed():
        return int(mb.shard_counters()[:, 2].sum())

    def batch(M, seed):
        g = torch.Generator().manual_seed(seed)
        a = torch.randint(0, n, (M,), generator=g, dtype=torch.int32)
        return B.MsgBatch(a.to(DEV), torch.ones(M, dtype=torch.int64, device=DEV), None, None, METHOD_COUNTER_ADD)

    # 1. unloaded rate: prefill ~3/4 of the rings, start the consumer, time the drain
    pre_n = (S * Q * 3) // 4
    cap_origins = 1 << 27
    out_v = torch.full((cap_origins,), -1, dtype=torch.int64, device=DEV)
    out_s = torch.full((cap_origins,), -1, dtype=torch.int32, device=DEV)
    pre = batch(pre_n, 1)
    mb.enqueue(pre, t, out_v, out_s, origin_base=0, live=True)
    torch.cuda.synchronize()
    actors = [pre.actor]
    origin = pre_n
    mb.start(state, out_v, out_s, blocks=2, max_s=30.0)
    t0 = time.perf_counter()
    while consumed() < pre_n and time.perf_counter() - t0 < 10:
        time.sleep(0.0005)
    r0 = pre_n / (time.perf_counter() - t0)
    # 2. sustained overload from two streams for > 1 s (paced at ~3x the unloaded rate)
    M = max(4096, int(3 * r0 * 0.002 / 2))  # per stream, every 2 ms
    reqs = [batch(M, 10 + k) for k in range(8)]
    streams = [torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)]
    c0, t_start = consumed(), time.perf_counter()
    k = 0
    while time.perf_counter() - t_start < 1.3 and origin + 2 * M <= cap_origins:
        for s in streams:
            r = reqs[k % len(reqs)]
            with torch.cuda.stream(s):
                mb.enqueue(r, t, out_v, out_s, origin_base=origin, live=True)
            actors.append(r.actor)
            origin += M
            k += 1
        time.sleep(0.002)
    c1, t_end = consumed(), time.perf_counter()
    r_over = (c1 - c0) / (t_end - t_start)
    for s in streams:
        s.synchronize()
    mb.stop()
    torch.cuda.synchronize()
    assert t_end - t_start > 1.0
    st = out_s[:origin]
    assert bool(((st == STATUS_OK) | (st == STATUS_OVERFLOW)).all())
    assert int((st == STATUS_OVERFLOW).sum()) > 0  # it really was overloaded
    assert r_over >= 0.8 * r0, f"consumer rate under overload {r_over / 1e6:.1f} M/s vs unloaded {r0 / 1e6:.1f} M/s"
    assert mb.stats()["holes"] == 0
    # exactly once: per actor, the OK replies are exactly 1..k and the state is k
    mbox = perm.to(DEV)[torch.cat(actors).long()]
    ok = st == STATUS_OK
    mo, vo = mbox[ok], out_v[:origin][ok]
    k_per = torch.bincount(mo, minlength=n)
    assert torch.equal(state, k_per)
    order = torch.argsort(mo * (1 << 40) + vo)
    start = torch.cumsum(k_per, 0) - k_per
    expect = torch.arange(mo.numel(), device=DEV) - start[mo[order]] + 1
    assert torch.equal(vo[order], expect)


# ---------------------------------------------------------------- sort kernels (mailbox_sort.hip)
@pytest.mark.parametrize("sort_mode", ["onepass", "twopass"])
@pytest.mark.parametrize("M", [5000, (1 << 20) + 333])
def test_sorted_mailbox_sort_modes_exact(sort_mode, M):
    """Every sort kernel (one pass, count + scatter)
    fills the same per-actor rings: exact replies, misses answered, rings
    consumed, no look-back timeout -- over Sends that reuse the rings."""
    n = 1 << 15
    t, _ = placed_table(n)
    mb = Mailboxes(DEV, shards=256, slots=1 << 14)
    g = torch.Generator().manual_seed(21)
    for rep in range(3):
        actor = torch.randint(0, n + 100, (M,), generator=g, dtype=torch.int32)
        a0 = torch.randint(-(1 << 31), 1 << 31, (M,), generator=g, dtype=torch.int64)
        a1 = torch.randint(-(1 << 20), 1 << 20, (M,), generator=g, dtype=torch.int64)
        req = B.MsgBatch(actor.to(DEV), a0.to(DEV), a1.to(DEV), None, METHOD_CALC_MULTIPLY)
        val, st = mb.send(req, t, None, sort_mode=sort_mode)
        torch.cuda.synchronize()
        known = actor < n
        st, val = st.cpu(), val.cpu()
        assert bool((st[known] == STATUS_OK).all()) and bool((st[~known] == STATUS_NO_ACTOR).all()), rep
        assert torch.equal(val[known], (a0 * a1)[known]), rep
        ctr = mb.shard_counters()
        assert (ctr[:, 0] == ctr[:, 2]).all()
    s = mb.stats()
    assert s["lookback_timeouts"] == 0 and s["holes"] == 0 and s["overflow"] == 0


def test_sorted_mailbox_onepass_ordered_fifo_and_spill():
    """The one-pass sort on the ordered path (full shard geometry, SeqFold chains
    audited exactly once and in message order per actor) and on a stateless
    batch whose rings overflow (spilled tiles drained in message order)."""
    n, M = 4096, 1 << 18
    t, perm = placed_table(n)
    state = torch.randint(0, 1 << 30, (n,), dtype=torch.int64, device=DEV)
    s0 = state.cpu().clone()
    mb = Mailboxes(DEV, shards=64, slots=1 << 14)
    req = fold_batch(M, n, 43)
    v, st = mb.send(req, t, state, sort_mode="onepass")
    torch.cuda.synchronize()
    ok, order = audit_fold(perm[req.actor.cpu().long()], req.a0.cpu(), v.cpu(), st.cpu(), s0, state.cpu())
    assert ok, order
    assert all(seq == sorted(seq) for seq in order.values())
    small = Mailboxes(DEV, shards=16, slots=4096)
    req2 = B.gen_requests(300_000, n, METHOD_CALC_MULTIPLY, seed=17, device=DEV)
    v2, st2 = small.send(req2, t, None, sort_mode="onepass")
    torch.cuda.synchronize()
    assert bool((st2 == STATUS_OK).all()) and torch.equal(v2, req2.a0 * req2.a1)
    s = small.stats()
    assert s["spilled"] > 0 and s["lookback_timeouts"] == 0 and s["processed"] == 300_000


def test_sorted_mailbox_onepass_graph_replays():
    """A captured one-pass Send replayed with new batches: its look-back tag comes
    from a device word the drain advances, so a replay never reads the previous
    replay's descriptors as its own."""
    n, M = 1 << 15, 1 << 19
    t, _ = placed_table(n)
    mb = Mailboxes(DEV, shards=256, slots=1 << 14)
    req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=1, device=DEV)
    val = torch.empty(M, dtype=torch.int64, device=DEV)
    st = torch.empty(M, dtype=torch.int32, device=DEV)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        mb.send(req, t, None, val, st, sort_mode="onepass")  # warm-up: workspaces grown outside the capture
    s.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        mb.send(req, t, None, val, st, sort_mode="onepass")
    for k in range(4):
        fresh = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=100 + k, device=DEV)
        req.actor.copy_(fresh.actor), req.a0.copy_(fresh.a0), req.a1.copy_(fresh.a1)
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        assert bool((st == STATUS_OK).all()) and torch.equal(val, req.a0 * req.a1), k
    assert mb.stats()["lookback_timeouts"] == 0


def test_sorted_mailbox_onepass_epoch_tag_wraps():
    """the one-pass look-back tag stays in the descriptor's
    24-bit field when its device counter passes 0xffffff -- every Send across
    the wrap sorts exactly and no look-back gives up."""
    n, M = 1 << 15, (1 << 20) + 333
    t, _ = placed_table(n)
    mb = Mailboxes(DEV, shards=256, slots=1 << 14)
    start = 0xFFFFFD
    mb._m.epoch_counter = start
    for k in range(4):  # tags 0xfffffe, 0xffffff, 1 (the counter's 0x1000000), 2
        req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=300 + k, device=DEV)
        val, st = mb.send(req, t, None, sort_mode="onepass")
        torch.cuda.synchronize()
        assert bool((st == STATUS_OK).all()) and torch.equal(val, req.a0 * req.a1), k
    assert mb._m.epoch_counter == start + 4
    assert mb.stats()["lookback_timeouts"] == 0


_ORD_REC8 = textwrap.dedent("""
    import json, os, sys, torch
    sys.path.insert(0, os.environ["PTYPE_ROOT"])
    sys.path.insert(0, os.path.join(os.environ["PTYPE_ROOT"], "tests"))
    from ptype_amd.ops import batch as B
    from ptype_amd.ops.mailbox import audit_fold
    from ptype_amd.ops.records import METHOD_SEQ_FOLD, STATUS_OK
    from ptype_amd.ops.table import RegistryTable, actor_keys
    from ptype_amd.parallel.exchange import ActorExchange
    dev = torch.device("cuda", 0)
    n, M = 65536, 4_300_000  # 1050 tiles: the one-pass sort (>= 1024 tiles), past the 512 that keep 16-B records
    t = RegistryTable(2 * n, device=dev)
    ids = torch.arange(n)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(5))
    t.upsert(actor_keys(ids), torch.zeros(n, dtype=torch.int32), perm.to(torch.int32))
    t.enable_directory(n)
    state = torch.randint(0, 1 << 30, (n,), dtype=torch.int64, device=dev)
    ex = ActorExchange(t, M, state=state)
    out = {}
    for rnd in range(3):
        g = torch.Generator().manual_seed(100 + rnd)
        actor = torch.randint(0, n, (M,), generator=g, dtype=torch.int32)
        # 16-bit arguments (8-B records), then arguments wider than the widths in force
        # (and later messages to the same actors): escape records keep their ring slots,
        # so nothing overflows and every actor still runs its messages in message order
        a0 = torch.randint(-30000, 30000, (M,), generator=g, dtype=torch.int64)
        if rnd == 2:
            a0[12345] = 1 << 40
            a0[200000:200064] = -(1 << 50)
        b = B.MsgBatch(actor.to(dev), a0.to(dev), None, None, METHOD_SEQ_FOLD)
        s0 = state.cpu().clone()
        r0 = ex.counters.resends
        v, st = ex.send_all(b)
        torch.cuda.synchronize()
        s1 = state.cpu().clone()
        ok, info = audit_fold(perm[actor.long()], a0, v.cpu(), st.cpu(), s0, s1)
        fifo = bool(ok) and all(seq == sorted(seq) for seq in info.values())
        out[rnd] = {"ok": bool(ok), "all_ok": bool((st == STATUS_OK).all()), "fifo": fifo,
                    "resends": int(ex.counters.resends - r0),
                    "rec_bytes": int(ex.mailboxes.last_record_bytes), "info": "" if ok else str(info)[:300]}
    print("RESULT " + json.dumps(out), flush=True)
""")


def test_mailbox_seqfold_in_8b_records_exactly_once_fifo():
    """Ordered Sends in 8-B records: each message's place in its tile rides through
    the ordered drain's reply stage, and a message whose argument outgrows the
    widths in force keeps its ring slot as an escape record (its fields in a side
    array) -- ADVICE r5: it used to overflow and be re-sent AFTER later messages of
    its actor had run.  Every actor's replies chain exactly once and in MESSAGE
    order (the audit's order checked against the indices), with no re-send round."""
    env = dict(os.environ, PTYPE_ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", _ORD_REC8], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    import json

    out = json.loads(line[0][7:])
    for rnd, o in out.items():
        assert o["ok"] and o["all_ok"] and o["fifo"], (rnd, o)
        assert o["resends"] == 0, (rnd, o)  # escapes: no message of an ordered Send overflows
    assert out["0"]["rec_bytes"] == 8 and out["2"]["rec_bytes"] == 8, out  # the ordered Sends really took 8-B records


@pytest.mark.parametrize("rec8", ["-1", "1"])
@pytest.mark.parametrize("M,slots", [(1 << 20, 1 << 16), (300_000, 2048)])
def test_arrival_fused_enqueue_drain_exact(M, slots, rec8, monkeypatch):
    """Arrival rings in one launch (mbx_arrival_fused_kernel: each block writes its
    tile's records into its ring run, then drains that run): stateless Multiply on
    rank byte routes (records carry actor ids; the presence map of route mode 4 is
    for batches past 512 tiles, test_arrival_fused_big_batch_presence_map) with
    unknown actors, exact -- in 16-B
    compact records (8-B ones per wave with tune mbox_rec8=1, the form of batches past
    512 tiles), and 32-B long ones for values past 32 bits; the
    commutative stateful CounterAdd through the same kernel (hash routes: every
    actor's count exact); with small rings the tiles past a ring's room spill and
    run from the batch.  Every ring drained afterwards."""
    from ptype_amd.ops.records import METHOD_COUNTER_ADD

    monkeypatch.setenv("PTYPE_TUNE", f"mbox_rec8={rec8}")
    n = 1 << 14
    t, _ = placed_table(n)
    mb = Mailboxes(DEV, shards=64, slots=slots)
    g = torch.Generator().manual_seed(21)
    actor = torch.randint(0, n + 700, (M,), generator=g, dtype=torch.int32).to(DEV)
    a0 = torch.randint(-(1 << 15), 1 << 15, (M,), generator=g, dtype=torch.int64).to(DEV)
    a1 = torch.randint(-(1 << 15), 1 << 15, (M,), generator=g, dtype=torch.int64).to(DEV)
    known = actor < n
    for k in range(3):
        if k == 2:  # a wide value in some tiles: those tiles take 16-B (or 32-B long) records
            a0 = a0.clone()
            a0[::40_000] = (1 << 40) + 7
            a1 = a1.clone()
            a1[5::70_000] = 1 << 21
        val, st = mb.send(B.MsgBatch(actor, a0, a1, None, METHOD_CALC_MULTIPLY), t, None, ordered=False,
                          sharding="arrival")
        torch.cuda.synchronize()
        assert mb.last_sharding == "arrival" and mb.last_route == 3  # (rank bytes: up to 512 tiles)
        assert mb.last_record_bytes == (8 if rec8 == "1" else 16)
        assert torch.equal(st, torch.where(known, STATUS_OK, STATUS_NO_ACTOR).to(torch.int32)), k
        assert torch.equal(val[known], (a0 * a1)[known]), k
    state = torch.zeros(n, dtype=torch.int64, device=DEV)
    ones = torch.ones(M, dtype=torch.int64, device=DEV)
    _, st = mb.send(B.MsgBatch(actor, ones, None, None, METHOD_COUNTER_ADD), t, state, ordered=False,
                    sharding="arrival")
    torch.cuda.synchronize()
    assert mb.last_route == 1  # (a stateful method keeps its mailbox route)
    assert torch.equal(st, torch.where(known, STATUS_OK, STATUS_NO_ACTOR).to(torch.int32))
    ref = torch.zeros(n, dtype=torch.int64)
    ref.index_add_(0, actor[known].long().cpu(), torch.ones(int(known.sum()), dtype=torch.int64))
    _, perm = placed_table(n)
    got = torch.empty(n, dtype=torch.int64)
    got[torch.arange(n)] = state.cpu()[perm]  # actor a lives in mailbox perm[a]
    assert torch.equal(got, ref)
    s = mb.stats()
    if slots < M // 64:
        assert s["spilled"] > 0, s
    assert s["overflow"] == 0, s
    ctr = mb.shard_counters()
    assert (ctr[:, 0] == ctr[:, 2]).all()


def test_exchange_takes_arrival_rings_for_small_stateless_sends():
    """World-1 ActorExchange with actor-sharded mailboxes (the default): a batch
    without ordered methods of up to 2 Mi messages takes the arrival rings (tune
    auto_arrival), an ordered one keeps the actor-sharded sort; replies exact."""
    n, M = 1 << 14, 400_000
    t, _ = placed_table(n)
    state = torch.zeros(n, dtype=torch.int64, device=DEV)
    ex = ActorExchange(t, M, delivery="mailbox", state=state)
    req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=5, device=DEV)
    val, st = ex.send(req)
    torch.cuda.synchronize()
    assert ex.mailboxes.last_sharding == "arrival"
    assert bool((st == STATUS_OK).all()) and torch.equal(val, req.a0 * req.a1)
    fold = fold_batch(M, n, seed=6)
    val, st = ex.send(fold)
    torch.cuda.synchronize()
    assert ex.mailboxes.last_sharding == "actor"
    assert bool((st == STATUS_OK).all())


@pytest.mark.parametrize("kept", [True, False])
def test_arrival_fused_big_batch_presence_map(kept):
    """A stateless batch past 512 tiles through the fused arrival Send: the
    directory's 2-bit presence map staged in LDS (route mode 4), 8-B records per
    wave; unknown ids (unregistered, past the directory) answered, replies exact --
    with the map the registry mirror keeps for this rank, and with one the Send
    folds itself (the mirror's is kept for another rank)."""
    n, M = 1 << 15, 5 << 20
    t = RegistryTable(4 * n, device=DEV)
    if not kept:
        t.set_presence_rank(1)
    ids = torch.cat([torch.arange(n), torch.arange(n + 100, n + 1100)])
    perm = torch.randperm(ids.numel(), generator=torch.Generator().manual_seed(31))
    t.upsert(actor_keys(ids), torch.zeros(ids.numel(), dtype=torch.int32), perm.to(torch.int32))
    t.enable_directory(n + 50)  # ids n..n+49: in the directory, unregistered; n+100..: hash probes
    g = torch.Generator().manual_seed(32)
    actor = torch.randint(0, n + 3000, (M,), generator=g, dtype=torch.int32).to(DEV)
    a0 = torch.randint(-(1 << 15), 1 << 15, (M,), generator=g, dtype=torch.int64).to(DEV)
    a1 = torch.randint(-(1 << 15), 1 << 15, (M,), generator=g, dtype=torch.int64).to(DEV)
    mb = Mailboxes(DEV, shards=256, slots=1 << 16)
    known = (actor < n) | ((actor >= n + 100) & (actor < n + 1100))
    for _ in range(2):
        val, st = mb.send(B.MsgBatch(actor, a0, a1, None, METHOD_CALC_MULTIPLY), t, None, ordered=False,
                          sharding="arrival")
        torch.cuda.synchronize()
        assert mb.last_route == 4 and mb.last_record_bytes == 8
        assert torch.equal(st, torch.where(known, STATUS_OK, STATUS_NO_ACTOR).to(torch.int32))
        assert torch.equal(val[known], (a0 * a1)[known])
    ctr = mb.shard_counters()
    assert (ctr[:, 0] == ctr[:, 2]).all()

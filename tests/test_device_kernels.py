"""Numerics of the hand-written gfx950 kernels vs plain PyTorch/NumPy references.

GPU tests compare each kernel against the CPU reference of the same op
(``ptype_amd/ops``); CPU tests pin the reference itself against hand-computed
expectations (so the references are not self-validating).
"""
import pytest
import torch

from ptype_amd import ops
from ptype_amd.ops import batch as B
from ptype_amd.ops.records import (METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD, METHOD_ECHO, METHOD_PRIME_CHECK,
                                   METHOD_RETRY_TEST, STATUS_FAILED, STATUS_NO_ACTOR, STATUS_OK, STATUS_OVERFLOW,
                                   make_requests, split_replies)
from ptype_amd.ops.table import RegistryTable, actor_keys


def _populate(table: RegistryTable, n_actors: int, R: int):
    ids = torch.arange(n_actors, dtype=torch.int64)
    table.upsert(actor_keys(ids), (ids % R).to(torch.int32), (ids // R).to(torch.int32))


# ----------------------------------------------------------------- CPU reference
def test_table_reference_roundtrip():
    t = RegistryTable(64, device="cpu")
    _populate(t, 40, 4)
    assert t.live == 40
    r, m = t.lookup(actor_keys(torch.tensor([0, 5, 39, 40])))
    assert r.tolist() == [0, 1, 3, -1]
    assert m.tolist() == [0, 1, 9, -1]
    found = t.delete(actor_keys(torch.tensor([5, 77])))
    assert found.tolist() == [True, False]
    assert t.live == 39 and t.tombstones == 1
    r, _ = t.lookup(actor_keys(torch.tensor([5, 6])))
    assert r.tolist() == [-1, 2]
    ent, exp = t.pack()
    assert ent.shape[0] == 39
    t.rebuild()
    assert t.live == 39 and t.tombstones == 0
    r, _ = t.lookup(actor_keys(torch.arange(40)))
    assert (r[torch.arange(40) != 5] >= 0).all() and r[5] == -1


def test_table_reference_sweep():
    t = RegistryTable(64, device="cpu")
    ids = torch.arange(8)
    t.upsert(actor_keys(ids), torch.zeros(8, dtype=torch.int32), ids.to(torch.int32),
             expiry=torch.tensor([0, 100, 200, 300, 0, 50, 500, 1000]))
    t.sweep(250)
    r, _ = t.lookup(actor_keys(ids))
    assert (r >= 0).tolist() == [True, False, False, True, True, False, True, True]


def _batch(actors, method, a0, a1=None, a2=None):
    t = lambda x: None if x is None else torch.as_tensor(x, dtype=torch.int64)
    m = method if isinstance(method, int) else torch.as_tensor(method, dtype=torch.int16)
    return B.MsgBatch(torch.as_tensor(actors, dtype=torch.int32), t(a0), t(a1), t(a2), m)


def _regions_equal(g, c, R, C, fmt):
    """Compare two request buffers on their defined words: headers + delivered records."""
    W = fmt.req_words(C)
    g, c = g.cpu(), c.cpu()
    for d in range(R):
        k = int(c[d * W])
        n = 4 + k * fmt.stride
        if not torch.equal(g[d * W:d * W + n], c[d * W:d * W + n]):
            return False
    return True


def _replies_equal(g, c, R, C):
    Wr = B.WireFormat.rep_words(C)
    g, c = g.cpu(), c.cpu()
    for d in range(R):
        k = int(c[d * Wr])
        gr, cr = g[d * Wr:(d + 1) * Wr], c[d * Wr:(d + 1) * Wr]
        if int(gr[0]) != k or not torch.equal(gr[4:4 + 2 * k], cr[4:4 + 2 * k]):
            return False
        if not torch.equal(gr[4 + 2 * C:].view(torch.uint8)[:k], cr[4 + 2 * C:].view(torch.uint8)[:k]):
            return False
    return True


@pytest.mark.parametrize("fmt", [B.FULL_FORMAT, B.WireFormat(2, False)])
def test_batch_reference_end_to_end(fmt):
    R, C = 3, 64
    t = RegistryTable(64, device="cpu")
    _populate(t, 12, R)
    req = _batch([0, 1, 2, 3, 4, 99], METHOD_CALC_MULTIPLY, [7, 2, 3, 4, 5, 6], [8, 3, 4, 5, 6, 7])
    send, perm, stats = B.route(req, t, R, C, fmt=fmt)
    W = fmt.req_words(C)
    assert send[0::W][:R].tolist() == [2, 2, 1]
    assert int(stats[B.STAT_NOMATCH]) == 1
    rep = B.dispatch(send, R, C, fmt=fmt)
    val, st = B.complete(rep, perm, C)
    assert val.tolist()[:5] == [56, 6, 12, 20, 30]
    assert st.tolist() == [STATUS_OK] * 5 + [STATUS_NO_ACTOR]


def test_wire_format_v2_layout():
    """Pin the v2 wire layout by hand: a calculator call is 5 words (20 B) with
    the uniform method in the slot header; replies are planar (i64 value + u8 status)."""
    fmt = B.WireFormat(2, False)
    assert fmt.stride == 5 and B.FULL_FORMAT.stride == 8 and B.WireFormat(3, False).stride == 7
    assert fmt.req_words(3) == 20 and B.WireFormat.rep_words(3) == 12
    t = RegistryTable(16, device="cpu")
    _populate(t, 4, 2)  # actor a -> rank a % 2, mbox a // 2
    req = _batch([3, 1, 2], METHOD_CALC_MULTIPLY, [-1, 5, 6], [1 << 33, 7, 8])
    send, perm, _ = B.route(req, t, 2, 3, rank_self=1, fmt=fmt)
    assert perm.tolist() == [3, 4, 0]  # d * C + pos; rank 1 gets actors 3 then 1 in message order
    r1 = send[20:40].tolist()
    assert r1[:4] == [2, 2, 1, (1 << 16) | METHOD_CALC_MULTIPLY]
    assert r1[4:9] == [1, -1, -1, 0, 2]  # mbox 1, a0 = -1 (lo, hi), a1 = 2^33 (lo 0, hi 2)
    rep = B.dispatch(send, 2, 3, fmt=fmt)
    assert rep.numel() == 2 * 12 and int(rep[12]) == 2
    assert rep[12 + 4:12 + 10].view(torch.int64)[:2].tolist() == [-(1 << 33), 35]
    val, st = B.complete(rep, perm, 3)
    assert val.tolist() == [-(1 << 33), 35, 48] and st.tolist() == [STATUS_OK] * 3
    with pytest.raises(ValueError):
        B.route(_batch([0], METHOD_ECHO, [1], [2], [3]), t, 2, 3, fmt=fmt)  # a2 does not fit


def test_batch_reference_overflow_and_handlers():
    R, C = 1, 8
    t = RegistryTable(16, device="cpu")
    _populate(t, 2, 1)
    state = torch.zeros(2, dtype=torch.int64)
    methods = [METHOD_COUNTER_ADD, METHOD_PRIME_CHECK] + [METHOD_ECHO] * 8
    req = _batch([0, 1] + [0] * 8, methods, [5, 2] + list(range(8)), [0, 10] + [0] * 8, [0, 21] + [0] * 8)
    send, perm, stats = B.route(req, t, R, C)
    rep = B.dispatch(send, R, C, state=state)
    val, st = B.complete(rep, perm, C)
    assert val.tolist()[:8] == [5, 3, 0, 1, 2, 3, 4, 5]  # counter 0+5, 21 = 3*7 -> first divisor 3
    assert st.tolist() == [STATUS_OK] * 8 + [STATUS_OVERFLOW] * 2
    assert int(stats[B.STAT_OVERFLOW]) == 2


def test_msgbatch_records_roundtrip():
    req = make_requests(torch.tensor([3, 4]), torch.tensor([METHOD_ECHO, METHOD_CALC_MULTIPLY]), torch.tensor([1, 2]),
                        torch.tensor([5, 6]), torch.tensor([7, 8]))
    b = B.MsgBatch.from_records(req)
    assert b.actor.tolist() == [3, 4] and b.method.tolist() == [METHOD_ECHO, METHOD_CALC_MULTIPLY]
    assert torch.equal(b.to_records(), req)


def test_retry_reference():
    v, s = B._handler_ref(torch.tensor([METHOD_RETRY_TEST] * 3), torch.tensor([0, 0, 0]), torch.tensor([2, 2, 2]),
                          torch.zeros(3, dtype=torch.int64), torch.zeros(3, dtype=torch.int64),
                          torch.zeros(1, dtype=torch.int64))
    assert s.tolist() == [STATUS_FAILED, STATUS_OK, STATUS_OK]
    assert v.tolist()[1:] == [2, 3]


# ----------------------------------------------------------------- GPU vs reference
@pytest.mark.gpu
def test_gpu_table_matches_reference():
    torch.manual_seed(0)
    n = 50_000
    g = RegistryTable(2 * n, device="cuda")
    c = RegistryTable(2 * n, device="cpu")
    keys = torch.randperm(10 * n)[:n].to(torch.int64) + 1
    ranks = torch.randint(0, 8, (n,), dtype=torch.int32)
    mbox = torch.randint(0, 1 << 20, (n,), dtype=torch.int32)
    g.upsert(keys.cuda(), ranks.cuda(), mbox.cuda())
    c.upsert(keys, ranks, mbox)
    torch.cuda.synchronize()
    assert g.live == n == c.live
    # same hash + same probing -> the slot images are identical for a single batch without duplicates
    probe = torch.cat([keys[::3], torch.arange(10 * n + 5, 10 * n + 1000)])
    rg, mg = g.lookup(probe.cuda())
    rc, mc = c.lookup(probe)
    assert torch.equal(rg.cpu(), rc) and torch.equal(mg.cpu(), mc)
    dk = keys[::7]
    fg = g.delete(dk.cuda())
    fc = c.delete(dk)
    assert torch.equal(fg.cpu(), fc)
    assert g.live == c.live and g.tombstones == c.tombstones
    rg, _ = g.lookup(keys.cuda())
    rc, _ = c.lookup(keys)
    assert torch.equal(rg.cpu(), rc)
    ent, _ = g.pack()
    assert ent.shape[0] == g.live
    assert set(ent[:, 0].cpu().tolist()) == set(keys[rc >= 0].tolist())
    g.rebuild()
    assert g.tombstones == 0
    rg2, _ = g.lookup(keys.cuda())
    assert torch.equal(rg2.cpu(), rc)


@pytest.mark.gpu
def test_gpu_table_sweep_and_snapshot():
    g = RegistryTable(1024, device="cuda")
    ids = torch.arange(300)
    exp = torch.where(ids % 3 == 0, torch.zeros_like(ids), ids * 10)
    g.upsert(actor_keys(ids).cuda(), torch.zeros(300, dtype=torch.int32).cuda(), ids.to(torch.int32).cuda(),
             exp.cuda())
    g.sweep(1500)
    r, _ = g.lookup(actor_keys(ids).cuda())
    expect = (exp == 0) | (exp >= 1500)
    assert torch.equal((r.cpu() >= 0), expect)
    h_ent, h_exp = g.snapshot_to_host()
    assert h_ent.is_pinned() and h_ent.shape[0] == int(expect.sum())
    g2 = RegistryTable(1024, device="cuda")
    g2.load_packed(h_ent, h_exp)
    r2, _ = g2.lookup(actor_keys(ids).cuda())
    assert torch.equal(r2.cpu(), r.cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("R,fmt", [(1, B.FULL_FORMAT), (2, B.WireFormat(2, False)), (8, B.WireFormat(2, False)),
                                   (8, B.WireFormat(3, True)), (3, B.WireFormat(2, True)),
                                   (16, B.WireFormat(2, False)), (20, B.WireFormat(2, False)),
                                   (64, B.WireFormat(2, False))])
def test_gpu_route_dispatch_complete(R, fmt):
    M, n_actors = 200_003, 4096
    C = B.stripe_capacity(M, R)
    g = RegistryTable(2 * n_actors, device="cuda")
    c = RegistryTable(2 * n_actors, device="cpu")
    _populate(g, n_actors, R)
    _populate(c, n_actors, R)
    req = B.gen_requests(M, n_actors, METHOD_CALC_MULTIPLY, seed=1234, device="cuda")
    ref = B.gen_requests(M, n_actors, METHOD_CALC_MULTIPLY, seed=1234, device="cpu")
    assert torch.equal(req.actor.cpu(), ref.actor) and torch.equal(req.a0.cpu(), ref.a0)
    assert torch.equal(req.a1.cpu(), ref.a1), "generator kernel differs from reference"
    send, perm, stats = B.route(req, g, R, C, rank_self=0, fmt=fmt)
    rsend, rperm, rstats = B.route(ref, c, R, C, rank_self=0, fmt=fmt)
    # deterministic stable placement: bit-identical to the CPU reference
    assert torch.equal(perm.cpu(), rperm)
    assert _regions_equal(send, rsend, R, C, fmt)
    assert stats.cpu().tolist()[:2] == rstats.tolist()[:2] == [0, 0]
    rep = B.dispatch(send, R, C, expected_per_rank=M // R, fmt=fmt)
    val, st = B.complete(rep, perm, C)
    rrep = B.dispatch(rsend, R, C, fmt=fmt)
    assert _replies_equal(rep, rrep, R, C)
    torch.cuda.synchronize()
    assert (st.cpu() == STATUS_OK).all()
    assert torch.equal(val.cpu(), ref.a0 * ref.a1)


@pytest.mark.gpu
@pytest.mark.parametrize("items,mode,pipe", [(0, 1, 0), (1, 0, -1), (2, 0, -1), (4, 0, -1), (8, 0, -1), (0, 0, 0),
                                             (2, 0, 0), (8, 0, 0)])
def test_gpu_route_directory_matches_hash_probe(items, mode, pipe):
    """K5b: routing through the dense directory is bit-identical to probing the
    hash table -- ids inside/outside the directory range, deleted ids, and an
    entry too wide for a route word (directory fallback to the probe)."""
    R, n_actors, M = 4, 6000, 100_000
    C = B.stripe_capacity(M, R)
    g = RegistryTable(2 * n_actors, device="cuda")
    c = RegistryTable(2 * n_actors, device="cpu")
    for t in (g, c):
        _populate(t, n_actors, R)
        t.delete(actor_keys(torch.arange(100, 200)))  # registered then removed
        t.upsert(actor_keys(torch.tensor([7])), torch.tensor([300]), torch.tensor([1]))  # rank 300: fallback
    g.enable_directory(4096)  # ids 4096.. probe the table
    req = B.gen_requests(M, n_actors + 50, METHOD_CALC_MULTIPLY, seed=99, device="cuda")  # some ids unregistered
    ref = B.gen_requests(M, n_actors + 50, METHOD_CALC_MULTIPLY, seed=99, device="cpu")
    try:
        ops.hip().set_route_tuning(items, mode, pipe)
        send, perm, stats = B.route(req, g, R, C)
    finally:
        ops.hip().set_route_tuning(0, 0, 0)
    rsend, rperm, rstats = B.route(ref, c, R, C)
    assert torch.equal(perm.cpu(), rperm)
    assert _regions_equal(send, rsend, R, C, B.FULL_FORMAT)
    assert stats.cpu().tolist()[:2] == rstats.tolist()[:2]
    assert rstats.tolist()[0] > 0  # misses were exercised
    # a later mutation invalidates the directory
    g.delete(actor_keys(torch.tensor([5])))
    c.delete(actor_keys(torch.tensor([5])))
    send, perm, _ = B.route(req, g, R, C)
    rsend, rperm, _ = B.route(ref, c, R, C)
    assert torch.equal(perm.cpu(), rperm)


@pytest.mark.gpu
@pytest.mark.parametrize("M,R,C,fmt", [(0, 3, 64, B.WireFormat(2, False)), (100, 2, 64, B.WireFormat(2, False)),
                                       (4096, 1, 5000, B.FULL_FORMAT), (70_001, 5, 9000, B.WireFormat(3, False)),
                                       (1_000_003, 8, 130_000, B.WireFormat(2, True))])
def test_gpu_route_single_pass_matches_three_pass(M, R, C, fmt):
    """The 3-pass route (default) and the single-pass look-back route produce the same bytes
    as the CPU reference: headers, records, perm, statistics -- including empty
    batches, sub-block batches, overflowing destinations and unknown actors."""
    n_actors = 3000
    g = RegistryTable(2 * n_actors, device="cuda")
    c = RegistryTable(2 * n_actors, device="cpu")
    _populate(g, n_actors, R)
    _populate(c, n_actors, R)
    g.enable_directory(n_actors)
    req = B.gen_requests(M, n_actors + 100, METHOD_CALC_MULTIPLY, seed=M + R, device="cuda")
    ref = B.gen_requests(M, n_actors + 100, METHOD_CALC_MULTIPLY, seed=M + R, device="cpu")
    if fmt.method_col:
        req.method = (req.actor % 3 + 1).to(torch.int16)
        ref.method = (ref.actor % 3 + 1).to(torch.int16)
    if fmt.nargs == 3:
        req.a2, ref.a2 = req.a1 * 3, ref.a1 * 3
    rsend, rperm, rstats = B.route(ref, c, R, C, fmt=fmt)
    outs = []
    for mode in (0, 1):
        ops.hip().set_route_tuning(0, mode)
        try:
            for _ in range(2):  # twice: the look-back epoch must advance cleanly between launches
                send, perm, stats = B.route(req, g, R, C, fmt=fmt)
        finally:
            ops.hip().set_route_tuning(0, 0)
        torch.cuda.synchronize()
        assert torch.equal(perm.cpu(), rperm), f"mode {mode}"
        assert _regions_equal(send, rsend, R, C, fmt), f"mode {mode}"
        assert stats.cpu().tolist()[:2] == rstats.tolist()[:2], f"mode {mode}"
        outs.append(stats.cpu().tolist()[:2])
    if M > 0:
        assert rstats.tolist()[0] > 0  # unknown actors were exercised


@pytest.mark.gpu
def test_gpu_route_overflow_and_unknown():
    R, C = 2, 1000
    g = RegistryTable(256, device="cuda")
    _populate(g, 100, R)
    actors = torch.cat([torch.zeros(1500, dtype=torch.int64), torch.tensor([555])])  # 1500 -> rank 0 (cap 1000)
    req = _batch(actors, METHOD_ECHO, torch.arange(1501))
    req = B.MsgBatch(req.actor.cuda(), req.a0.cuda(), None, None, METHOD_ECHO)
    send, perm, stats = B.route(req, g, R, C)
    rep = B.dispatch(send, R, C)
    val, st = B.complete(rep, perm, C)
    st = st.cpu()
    # stable order: the first C messages are delivered, the rest overflow to the next epoch
    assert st[:1000].eq(STATUS_OK).all() and st[1000:1500].eq(STATUS_OVERFLOW).all()
    assert int(st[1500]) == STATUS_NO_ACTOR
    assert stats.cpu().tolist()[:2] == [1, 500]
    assert torch.equal(val.cpu()[:1000], torch.arange(1000))


@pytest.mark.gpu
def test_gpu_stateful_handlers_match_reference():
    R, C = 1, 8192
    g = RegistryTable(64, device="cuda")
    _populate(g, 4, 1)
    n = 1000
    actors = torch.arange(n) % 4
    b = _batch(actors, METHOD_COUNTER_ADD, torch.ones(n, dtype=torch.int64))
    req = B.MsgBatch(b.actor.cuda(), b.a0.cuda(), None, None, METHOD_COUNTER_ADD)
    state = torch.zeros(4, dtype=torch.int64, device="cuda")
    send, perm, _ = B.route(req, g, R, C)
    rep = B.dispatch(send, R, C, state=state)
    val, st = B.complete(rep, perm, C)
    assert state.cpu().tolist() == [250] * 4
    # per-actor values are a permutation of 1..250 (arrival order is the device's)
    v = val.cpu()
    for a in range(4):
        assert sorted(v[actors == a].tolist()) == list(range(1, 251))
    # prime check vs reference
    tgt = torch.tensor([97, 91, 221, 1000003, 49])
    b = _batch(torch.zeros(5, dtype=torch.int64), METHOD_PRIME_CHECK, torch.full((5,), 2), torch.full((5,), 1 << 40), tgt)
    req = B.MsgBatch(b.actor.cuda(), b.a0.cuda(), b.a1.cuda(), b.a2.cuda(), METHOD_PRIME_CHECK)
    send, perm, _ = B.route(req, g, R, C)
    val, st = B.complete(B.dispatch(send, R, C), perm, C)
    assert val.cpu().tolist() == [97, 7, 13, 1000003, 7]


@pytest.mark.gpu
def test_gpu_device_server_latency_path():
    import time

    state = torch.zeros(8, dtype=torch.int64, device="cuda")
    srv = ops.hip().DeviceServer(0, 1024, state.data_ptr(), 8, 0, 50.0, 20.0)
    try:
        v, s, a = srv.call(METHOD_CALC_MULTIPLY, 0, 7, 8)
        assert (v, s) == (56, STATUS_OK)
        # stateful retry actor: fails until count >= 3
        outs = [srv.call(METHOD_RETRY_TEST, 2, 3)[1] for _ in range(4)]
        assert outs == [STATUS_FAILED, STATUS_FAILED, STATUS_OK, STATUS_OK]
        # batched submit through pinned records
        n = 5000
        req = make_requests(torch.arange(n) % 8, METHOD_CALC_MULTIPLY, torch.arange(n), torch.full((n,), 3)).pin_memory()
        rep = torch.zeros(n, 2, dtype=torch.int64).pin_memory()
        srv.call_many(req.data_ptr(), rep.data_ptr(), n)
        val, st, _ = split_replies(rep)
        assert torch.equal(val, torch.arange(n) * 3) and (st == 0).all()
        # idle exit + transparent relaunch
        time.sleep(0.3)
        assert not srv.running
        assert srv.call(METHOD_ECHO, 1, 42)[0] == 42
        assert srv.launches >= 2
        lat = []
        for i in range(2000):
            t0 = time.perf_counter()
            srv.call(METHOD_CALC_MULTIPLY, i % 8, i, 2)
            lat.append(time.perf_counter() - t0)
        lat.sort()
        print("device-server p50 RTT us", lat[len(lat) // 2] * 1e6, "p99", lat[int(len(lat) * 0.99)] * 1e6)
    finally:
        srv.close()


@pytest.mark.gpu
def test_gpu_device_server_timeout_does_not_wedge_ring():
    """a timed-out call must not hand its slot to the next occupant while
    the dispatcher may still read it.  One slow call (Prime.Check with a per-candidate
    delay) times out; the next `ring` calls -- the last one reusing the timed-out
    slot -- all complete, and the late reply is taken over, not lost."""
    from ptype_amd.ops.records import METHOD_PRIME_CHECK

    ring = 64
    state = torch.zeros(8, dtype=torch.int64, device="cuda")
    srv = ops.hip().DeviceServer(0, ring, state.data_ptr(), 8, 20_000, 200.0, 20.0)  # 20 ms per candidate
    try:
        with pytest.raises(RuntimeError, match="timeout"):
            srv.call(METHOD_PRIME_CHECK, 0, 2, 10, 101, 0.05)  # 8 candidates x 20 ms > 50 ms
        for i in range(ring + 8):
            v, s, _ = srv.call(METHOD_CALC_MULTIPLY, i % 8, i, 5, 0, 10.0)
            assert (v, s) == (5 * i, STATUS_OK)
    finally:
        srv.close()


def test_wire_sizes_match_kernels():
    """The Python geometry and the launchers' must agree (the all-to-all splits on it)."""
    h = ops.hip()
    for C in (1, 3, 64, 1000, 123457):
        for nargs in (1, 2, 3):
            for mc in (False, True):
                assert h.wire_req_words(C, nargs, mc) == B.WireFormat(nargs, mc).req_words(C)
        assert h.wire_rep_words(C) == B.WireFormat.rep_words(C)


@pytest.mark.gpu
def test_gpu_send_graph_replay():
    """hipGraph capture of generator + Send: every replay routes a fresh batch."""
    from ptype_amd.parallel.exchange import ActorExchange

    n_actors, M = 4096, 300_000
    g = RegistryTable(2 * n_actors, device="cuda")
    _populate(g, n_actors, 1)
    g.enable_directory(n_actors)
    state = torch.zeros(n_actors, dtype=torch.int64, device="cuda")
    ex = ActorExchange(g, M, state=state)
    req = B.gen_requests(M, n_actors, METHOD_CALC_MULTIPLY, seed=1, device="cuda")
    val = torch.empty(M, dtype=torch.int64, device="cuda")
    st = torch.empty(M, dtype=torch.int32, device="cuda")
    seed_t = torch.tensor([11], dtype=torch.int64, device="cuda")

    def prologue():
        B.gen_requests(M, n_actors, METHOD_CALC_MULTIPLY, device="cuda", out=req, seed_tensor=seed_t)
        seed_t.add_(1)

    graph = ex.capture(req, val, st, prologue=prologue)
    seen = []
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        assert bool((st == STATUS_OK).all()) and torch.equal(val, req.a0 * req.a1)
        seen.append(req.actor[:8].cpu().tolist())
    assert seen[0] != seen[1] != seen[2]
    assert ex.stats().sent >= 3 * M


@pytest.mark.gpu
def test_gpu_send_graph_repeat():
    """A graph holding 3 whole steps (prologue + Send each): one replay advances the
    generator 3 times, and the last step's replies are the ones left in the outputs."""
    from ptype_amd.parallel.exchange import ActorExchange

    n_actors, M = 2048, 100_000
    g = RegistryTable(2 * n_actors, device="cuda")
    _populate(g, n_actors, 1)
    g.enable_directory(n_actors)
    ex = ActorExchange(g, M, state=torch.zeros(n_actors, dtype=torch.int64, device="cuda"))
    req = B.gen_requests(M, n_actors, METHOD_CALC_MULTIPLY, seed=1, device="cuda")
    val = torch.empty(M, dtype=torch.int64, device="cuda")
    st = torch.empty(M, dtype=torch.int32, device="cuda")
    seed_t = torch.tensor([100, 101, 102], dtype=torch.int64, device="cuda")
    steps = []

    def prologue(j):
        steps.append(j)
        B.gen_requests(M, n_actors, METHOD_CALC_MULTIPLY, device="cuda", out=req, seed_tensor=seed_t[j:j + 1])
        if j == 2:
            seed_t.add_(3)

    graph = ex.capture(req, val, st, prologue=prologue, repeat=3)
    assert steps[-3:] == [0, 1, 2]  # the captured body: steps 0, 1, 2 of a replay
    s0 = int(seed_t[2].item())
    sent0 = ex.stats().sent
    graph.replay()
    torch.cuda.synchronize()
    assert int(seed_t[2].item()) == s0 + 3
    ref = B.gen_requests(M, n_actors, METHOD_CALC_MULTIPLY, seed=s0, device="cuda")  # the replay's last batch
    assert torch.equal(req.actor, ref.actor) and torch.equal(val, ref.a0 * ref.a1) and bool((st == STATUS_OK).all())
    assert ex.stats().sent - sent0 == 3 * M


def test_no_kernel_spills_to_scratch():
    """Every gfx950 kernel compiles without scratch (private memory): twice a
    silent spill cost 3x (an indexed probe group) and 56 MB of HBM writes per
    epoch (the address of a by-value kernel argument).  Reads the resource-usage
    remarks the build keeps next to the objects."""
    from ptype_amd import _build

    _build.build_hip()
    res = _build.kernel_resources()
    assert len(res) >= 20, "resource remarks missing (hipcc -Rpass-analysis=kernel-resource-usage)"
    spills = {k: v for k, v in res.items() if v.get("ScratchSize", 0) > 0}
    assert not spills, spills
    low = {k: v for k, v in res.items() if "route" in k and v.get("Occupancy", 8) < 4}
    assert not low, low


@pytest.mark.gpu
@pytest.mark.parametrize("R,self_rank,mode", [(1, 0, 0), (3, 1, 0), (8, 5, 0), (3, 2, 1)])
def test_gpu_direct_completion_matches(R, self_rank, mode):
    """Direct completion (own slot replies straight into the outputs, statuses of
    unknown / overflowed messages written by the route) gives exactly the
    outputs of the staged path -- both route algorithms."""
    n_actors, M = 5000, 200_000
    C = B.stripe_capacity(M, R) // 2 if R > 1 else M  # force overflow on multi-rank cases
    g = RegistryTable(2 * n_actors, device="cuda")
    _populate(g, n_actors, R)
    g.enable_directory(n_actors)
    req = B.gen_requests(M, n_actors + 50, METHOD_CALC_MULTIPLY, seed=R * 7 + self_rank, device="cuda")
    fmt = B.WireFormat(2, False)
    ops.hip().set_route_tuning(0, mode)
    try:
        send, perm, _ = B.route(req, g, R, C, rank_self=self_rank, fmt=fmt)
        rep = B.dispatch(send, R, C, fmt=fmt, rank_self=self_rank)
        ref_val, ref_st = B.complete(rep, perm, C)
        val = torch.full((M,), -7, dtype=torch.int64, device="cuda")
        st = torch.full((M,), -7, dtype=torch.int32, device="cuda")
        src = torch.empty(C, dtype=torch.int32, device="cuda")
        send2, perm2, _ = B.route(req, g, R, C, rank_self=self_rank, fmt=fmt, direct=(val, st, src))
        rep2 = B.dispatch(send2, R, C, fmt=fmt, direct=(val, st, src), rank_self=self_rank)
        B.complete(rep2, perm2, C, val, st, direct=True)
    finally:
        ops.hip().set_route_tuning(0, 0)
    torch.cuda.synchronize()
    assert torch.equal(val, ref_val) and torch.equal(st, ref_st)
    assert int((perm2 == -3).sum()) > 0 and bool((st != -7).all())


@pytest.mark.gpu
@pytest.mark.parametrize("W", [1, 3, 8])
def test_gpu_affine_placement_route(W):
    """Verified strided placement: the route computes route words (no directory
    gathers) while every id sits at (id % W, id // W); a re-homed or removed actor
    drops it back to the directory.  Bit-identical to the CPU reference throughout."""
    n_actors, M = 6000, 150_000
    C = B.stripe_capacity(M, W)
    g = RegistryTable(2 * n_actors, device="cuda")
    c = RegistryTable(2 * n_actors, device="cpu")
    _populate(g, n_actors, W)
    _populate(c, n_actors, W)
    g.enable_directory(n_actors, affine_world=W)
    req = B.gen_requests(M, n_actors + 70, METHOD_CALC_MULTIPLY, seed=W, device="cuda")
    ref = B.gen_requests(M, n_actors + 70, METHOD_CALC_MULTIPLY, seed=W, device="cpu")
    fmt = B.WireFormat(2, False)

    def check():
        send, perm, st = B.route(req, g, W, C, fmt=fmt)
        rsend, rperm, rst = B.route(ref, c, W, C, fmt=fmt)
        assert torch.equal(perm.cpu(), rperm) and _regions_equal(send, rsend, W, C, fmt)
        assert st.cpu().tolist()[:2] == rst.tolist()[:2]

    check()
    assert g.affine == W
    for t in (g, c):  # re-home one actor: the rule no longer holds
        t.upsert(actor_keys(torch.tensor([10])), torch.tensor([(10 + 1) % W]), torch.tensor([999]))
    check()
    assert g.affine == 0


@pytest.mark.gpu
@pytest.mark.parametrize("chunks", [1, 3])
def test_gpu_exactly_once_1m(chunks):
    """1M CounterAdd(+1) messages through the exchange: every
    actor's state equals the number of messages sent to it, and the replies it
    returned are exactly 1..count -- nothing lost, duplicated or mis-replied."""
    from ptype_amd.parallel.exchange import ActorExchange

    n_actors, M = 4096, 1 << 20
    g = RegistryTable(2 * n_actors, device="cuda")
    _populate(g, n_actors, 1)
    g.enable_directory(n_actors, affine_world=1)
    state = torch.zeros(n_actors, dtype=torch.int64, device="cuda")
    ex = ActorExchange(g, M, chunks=chunks, state=state)
    actors = torch.randint(0, n_actors, (M,), generator=torch.Generator().manual_seed(chunks)).to(torch.int32)
    req = B.MsgBatch(actors.cuda(), torch.ones(M, dtype=torch.int64, device="cuda"), None, None, METHOD_COUNTER_ADD)
    val, st = ex.send(req)
    torch.cuda.synchronize()
    assert bool((st == STATUS_OK).all())
    counts = torch.bincount(actors.long(), minlength=n_actors)
    assert torch.equal(state.cpu(), counts)
    # per actor, the returned post-increment values are a permutation of 1..count
    order = torch.argsort(actors.long() * (M + 1) + val.cpu())
    a_sorted, v_sorted = actors.long()[order], val.cpu()[order]
    first = torch.cumsum(counts, 0) - counts
    rank_in_actor = torch.arange(M) - first[a_sorted]
    assert torch.equal(v_sorted, rank_in_actor + 1)


@pytest.mark.gpu
@pytest.mark.parametrize("mfma", [False, True])
def test_gpu_records_to_soa(mfma):
    """AoS -> SoA on the device, both the dwordx4 copy and the MFMA byte
    transposition, equal the CPU split (including negative / high-bit values and
    a tail that is not a multiple of the 16-record MFMA tile)."""
    M = 100_003
    g = torch.Generator().manual_seed(3)
    actor = torch.randint(0, 1 << 31, (M,), generator=g)
    method = torch.randint(0, 1 << 15, (M,), generator=g)
    a0, a1, a2 = (torch.randint(-(1 << 62), 1 << 62, (M,), generator=g) for _ in range(3))
    req = make_requests(actor, method, a0, a1, a2)
    ref = B.MsgBatch.from_records(req)
    out = B.MsgBatch.from_records(req.cuda(), mfma=mfma)
    torch.cuda.synchronize()
    assert torch.equal(out.actor.cpu(), ref.actor) and torch.equal(out.method.cpu(), ref.method)
    assert torch.equal(out.a0.cpu(), ref.a0) and torch.equal(out.a1.cpu(), ref.a1) and torch.equal(out.a2.cpu(), ref.a2)


@pytest.mark.gpu
def test_prime_gather_kernel_matches_reference():
    """csrc/hip/optimus.hip: the device gather (one wave per target, early exit at
    the first deciding reply) equals the host reference, failed statuses included."""
    import torch

    from ptype_amd.models.optimus import FanOut, gather_ref
    from ptype_amd.ops import batch as B
    from ptype_amd.ops.records import METHOD_PRIME_CHECK

    g = torch.Generator().manual_seed(4)
    targets = torch.randint(2, 200_000, (3000,), generator=g)
    f = FanOut(targets, 4096, "cuda")
    b = f.batch
    val, st = B._handler_ref(torch.full((f.M,), METHOD_PRIME_CHECK), b.actor.long().cpu(), b.a0.cpu(), b.a1.cpu(),
                             b.a2.cpu(), None)
    st = st.to(torch.int32)
    st[torch.randint(0, f.M, (50,), generator=g)] = 3  # a few failed ranges
    ans, status = f.gather(val.cuda(), st.cuda())
    ref_a, ref_s = gather_ref(val, st, f.first.cpu(), f.n.cpu(), f.targets.cpu())
    torch.cuda.synchronize()
    ok = ref_s == 0
    assert torch.equal(status.cpu(), ref_s) and torch.equal(ans.cpu()[ok], ref_a[ok])

"""Sorted exchange (csrc/hip/exchange_sorted.hpp) on MI355X: the multi-GPU Send
with mailbox delivery, run on one GPU as R in-process ranks (FakeComm: one host
thread + stream per rank, the all-to-alls as device copies between them).

* calculator replies exact across Sends 0-1 (start-up wide layout) and 2+
  (layout and capacity agreed two Sends earlier -- no host wait per Send);
* ordered SeqFold traffic from every rank to every rank's actors: every actor's
  replies chain exactly once (audit_fold) and each (sender, actor) pair ran in
  message order;
* a message wider than the layout in force is answered STATUS_OVERFLOW (its slot
  carries a null record) and send_all re-sends it until the agreed layout grows.
"""
import json
import os
import subprocess
import sys
import textwrap
import threading

import pytest
import torch

from ptype_amd.ops import batch as B
from ptype_amd.ops import hip
from ptype_amd.ops.mailbox import audit_fold
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_SEQ_FOLD, STATUS_OK, STATUS_OVERFLOW
from ptype_amd.ops.table import RegistryTable, actor_keys
from ptype_amd.parallel.exchange import ActorExchange

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run_ranks(R, body, timeout=240):
    fc = hip().FakeComm(R)
    res, errors = [None] * R, []
    start = threading.Barrier(R)

    def run(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                res[r] = body(r, fc, start, s)
        except BaseException as e:  # noqa: BLE001
            errors.append((r, repr(e)))

    ths = [threading.Thread(target=run, args=(r,)) for r in range(R)]
    [t.start() for t in ths]
    [t.join(timeout=timeout) for t in ths]
    assert not errors, errors
    return res


def _table(n, R):
    tab = RegistryTable(2 * n, device="cuda")
    ids = torch.arange(n)
    g = torch.Generator().manual_seed(99)
    slot = torch.randperm(n, generator=g)  # random placement: routes read the mirror
    tab.upsert(actor_keys(ids), (slot % R).to(torch.int32), (slot // R).to(torch.int32))
    tab.enable_directory(n)
    return tab, slot


@pytest.mark.parametrize("R,chunks", [(2, 1), (3, 2), (4, 2)])
def test_sorted_exchange_calculator_exact_across_layouts(R, chunks):
    n, M = 8192, 100_000

    def body(r, fc, start, s):
        tab, _ = _table(n, R)
        st = torch.zeros(n // R + 1, dtype=torch.int64, device="cuda")
        ex = ActorExchange(tab, M, chunks=chunks, state=st, fake=(fc, r), delivery="mailbox", mailbox_ordered=False)
        start.wait()
        wires = []
        for k in range(5):
            req = B.gen_requests(M - 777 * r, n, METHOD_CALC_MULTIPLY, seed=40 + 7 * r + k, device="cuda")
            v, sts = ex.send(req)
            s.synchronize()
            assert bool((sts == STATUS_OK).all()), (k, int((sts != STATUS_OK).sum()))
            assert torch.equal(v, req.a0 * req.a1)
            wires.append(dict(ex.last_wire))
        return wires

    res = _run_ranks(R, body)
    for wires in res:
        assert wires[0]["engine"] == "sorted" and not wires[0]["agreed"] and wires[0]["S"] == 8
        assert wires[2]["agreed"] and wires[2]["spec_from"] == 0 and wires[4]["spec_from"] == 2
        assert wires[2]["S"] <= 2 and wires[2]["vb"] == 4  # 16-bit args, 17-bit mailboxes: 8-B records
    assert len({w[3]["C"] for w in res}) == 1  # every rank derived the same geometry


@pytest.mark.parametrize("R", [2, 4])
def test_sorted_exchange_ordered_seqfold_fifo_per_sender(R):
    n, M = 4096, 60_000

    def fold(M, seed):
        g = torch.Generator().manual_seed(seed)
        return B.MsgBatch(torch.randint(0, n, (M,), generator=g, dtype=torch.int32).cuda(),
                          torch.randint(-(1 << 20), 1 << 20, (M,), generator=g, dtype=torch.int64).cuda(),
                          None, None, METHOD_SEQ_FOLD)

    states0 = [torch.randint(0, 1 << 30, (n // R + 1,), dtype=torch.int64,
                             generator=torch.Generator().manual_seed(r)) for r in range(R)]

    def body(r, fc, start, s):
        tab, slot = _table(n, R)
        st = states0[r].cuda()
        ex = ActorExchange(tab, M, chunks=2, state=st, fake=(fc, r), delivery="mailbox")
        start.wait()
        out = []
        for k in range(3):  # Sends 0-1 wide, Send 2 agreed
            req = fold(M, 500 + 10 * r + k)
            v, sts = ex.send(req)
            s.synchronize()
            out.append((req.actor.cpu().long(), req.a0.cpu(), v.cpu(), sts.cpu()))
        return out, st.cpu(), slot

    res = _run_ranks(R, body)
    slot = res[0][2]
    P = n // R + 1
    # global mailbox key of an actor: owner rank * P + local mailbox
    key_of = lambda a: (slot[a] % R) * P + slot[a] // R  # noqa: E731
    before = torch.cat(states0)
    after = torch.cat([x[1] for x in res])
    actor = torch.cat([torch.cat([o[k][0] for k in range(3)]) for o, _, _ in res])
    a0 = torch.cat([torch.cat([o[k][1] for k in range(3)]) for o, _, _ in res])
    v = torch.cat([torch.cat([o[k][2] for k in range(3)]) for o, _, _ in res])
    sts = torch.cat([torch.cat([o[k][3] for k in range(3)]) for o, _, _ in res])
    ok, order = audit_fold(key_of(actor), a0, v, sts, before, after)
    assert ok, order
    # per (sender, actor): message order (senders' messages are concatenated rank-major, Send-major)
    sizes = [sum(len(o[k][0]) for k in range(3)) for o, _, _ in res]
    bounds = torch.cumsum(torch.tensor([0] + sizes), 0)
    for x, seq in list(order.items())[:256]:
        for r in range(R):
            mine = [i for i in seq if bounds[r] <= i < bounds[r + 1]]
            assert mine == sorted(mine), f"actor {x}: sender {r}'s messages out of order"


def test_sorted_exchange_zipf_skew_moves_per_pair_prefixes():
    """under Zipf(1.1) load one destination is hot; the agreed
    per-(sender, destination) capacities move each region's used prefix
    (grouped send / recv) instead of every pair at the hot pair's size.  Replies
    exact, no re-send once the agreement applies, fewer words than padding."""
    R, n, M = 4, 8192, 120_000

    def body(r, fc, start, s):
        tab, _ = _table(n, R)
        st = torch.zeros(n // R + 1, dtype=torch.int64, device="cuda")
        ex = ActorExchange(tab, M, chunks=1, state=st, fake=(fc, r), delivery="mailbox", mailbox_ordered=False)
        start.wait()
        wires, resends = [], []
        for k in range(7):
            req = B.gen_zipf_requests(M, n, 1.1, seed=900 + 13 * r + k, device="cuda")
            before = ex.counters.resends
            v, sts = ex.send_all(req)
            s.synchronize()
            assert bool((sts == STATUS_OK).all()), (k, int((sts != STATUS_OK).sum()))
            assert torch.equal(v, req.a0 * req.a1), k
            wires.append(dict(ex.last_wire))
            resends.append(ex.counters.resends - before)
        return wires, resends

    res = _run_ranks(R, body)
    for wires, resends in res:
        w = wires[-1]
        assert w["pairs"], w
        assert max(w["cap_in"]) > 1.2 * min(w["cap_in"]) or max(w["cap_out"]) > 1.2 * min(w["cap_out"]), w
        padded = R * (w["C"] * w["S"])
        assert w["req_words"] < 0.9 * padded, (w["req_words"], padded)
        assert sum(resends[4:]) == 0, resends
    caps = [tuple(x[0][-1]["cap_out"]) for x in res]
    ins = [tuple(x[0][-1]["cap_in"]) for x in res]
    for p in range(R):  # sender p's capacity toward q is what q expects from p
        for q in range(R):
            assert caps[p][q] == ins[q][p]


def test_sorted_exchange_too_wide_is_overflow_then_resent():
    R, n, M = 2, 4096, 20_000

    def body(r, fc, start, s):
        tab, _ = _table(n, R)
        st = torch.zeros(n // R + 1, dtype=torch.int64, device="cuda")
        ex = ActorExchange(tab, M, chunks=1, state=st, fake=(fc, r), delivery="mailbox", mailbox_ordered=False)
        start.wait()
        for k in range(3):  # settle a narrow layout (16-bit arguments)
            req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=3 + k + 10 * r, device="cuda")
            ex.send(req)
        s.synchronize()
        wide = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=77 + r, device="cuda")
        wide.a0[::100] = 1 << 40  # 1 % of the messages need 42-bit arguments
        v, sts = ex.send(wide)
        s.synchronize()
        first = sts.clone()
        v, sts = ex.send_all(wide)  # re-sends until the agreed layout holds them
        s.synchronize()
        return first.cpu(), v.cpu(), sts.cpu(), (wide.a0 * wide.a1).cpu(), ex.counters.resends

    for first, v, sts, ref, resends in _run_ranks(R, body):
        assert int((first == STATUS_OVERFLOW).sum()) == len(first[::100])
        assert bool((sts == STATUS_OK).all()) and torch.equal(v, ref) and resends >= 1


def test_sorted_exchange_onepass_epoch_tag_wraps_in_a_subprocess():
    """the sorted exchange's one-pass look-back sort (tune sx_sort=1)
    across its epoch counter's 24-bit tag wrap: exact replies, no stalled look-back."""
    code = textwrap.dedent("""
        import sys, torch
        sys.path.insert(0, sys.argv[1])
        sys.path.insert(0, sys.argv[1] + "/tests")
        from test_sorted_exchange_gpu import _run_ranks, _table
        from ptype_amd.ops import batch as B
        from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, STATUS_OK
        from ptype_amd.parallel.exchange import ActorExchange
        R, n, M = 2, 8192, 100_000
        def body(r, fc, start, s):
            tab, _ = _table(n, R)
            st = torch.zeros(n // R + 1, dtype=torch.int64, device="cuda")
            ex = ActorExchange(tab, M, chunks=1, state=st, fake=(fc, r), delivery="mailbox", mailbox_ordered=False)
            req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=5 + r, device="cuda")
            ex.send(req)  # builds the engine
            s.synchronize()
            ex._sorted.epoch_counter = 0xFFFFFD
            start.wait()
            for k in range(4):
                req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=60 + 5 * r + k, device="cuda")
                v, sts = ex.send(req)
                s.synchronize()
                assert bool((sts == STATUS_OK).all()) and torch.equal(v, req.a0 * req.a1), (r, k)
            assert ex._sorted.epoch_counter == 0xFFFFFD + 4
            assert ex.stats().failed == 0  # (raises on a stalled look-back)
            return True
        assert all(_run_ranks(R, body))
        print("SUBPROCESS-OK")
    """)
    env = dict(os.environ, PTYPE_TUNE="sx_sort=1")
    p = subprocess.run([sys.executable, "-c", code, ROOT], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0 and "SUBPROCESS-OK" in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])


_GRAPH_SCRIPT = textwrap.dedent("""
    import json, os, sys, torch, torch.distributed as dist
    sys.path.insert(0, os.environ["PTYPE_ROOT"])
    from ptype_amd.ops import batch as B
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, STATUS_OK
    from ptype_amd.ops.table import RegistryTable, actor_keys
    from ptype_amd.parallel.exchange import ActorExchange
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from ptype_amd.parallel.native_group import solo_group
    G = solo_group(dev)  # the compiled DataPlane's RCCL communicator, world 1 (collectives forced on)
    n, M = 1 << 15, 1 << 20
    t = RegistryTable(2 * n, device=dev)
    ids = torch.arange(n)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(3))
    t.upsert(actor_keys(ids), torch.zeros(n, dtype=torch.int32), perm.to(torch.int32))
    t.enable_directory(n, affine_world=1)
    ex = ActorExchange(t, M, chunks=2, delivery="mailbox", mailbox_ordered=False, group=G)
    assert ex.force_collectives and ex._use_sorted()
    req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=1, device=dev)
    val = torch.empty(M, dtype=torch.int64, device=dev)
    st = torch.empty(M, dtype=torch.int32, device=dev)
    for _ in range(3):  # past the start-up layout: Send 2 runs on an agreed one
        ex.send(req, val, st)
    torch.cuda.synchronize()
    print("warm", flush=True, file=sys.stderr)
    seed = torch.tensor([11], dtype=torch.int64, device=dev)
    def prologue():
        B.gen_requests(M, n, METHOD_CALC_MULTIPLY, device=dev, out=req, seed_tensor=seed)
        seed.add_(1)
    g = ex.capture(req, val, st, prologue=prologue, allow_collectives=True)
    print("captured", flush=True, file=sys.stderr)
    oks = []
    for k in range(4):  # every replay: new requests, a whole sorted-exchange Send with RCCL all-to-alls
        g.replay()
        torch.cuda.synchronize()
        print("replay", k, flush=True, file=sys.stderr)
        oks.append(bool((st == STATUS_OK).all()) and bool(torch.equal(val, req.a0 * req.a1)))
    w = ex.last_wire
    print("RESULT " + json.dumps({"ok": oks, "engine": w["engine"], "agreed": bool(w["agreed"]), "S": int(w["S"])}))
    G.close()
""")


@pytest.mark.gpu
def test_sorted_exchange_step_captures_into_a_hipgraph():
    """the N > 1 Send path (the sorted exchange: packed wire-v3
    records, comm-stream fork / join per chunk, the layout in force -- no host
    wait) captured into a hipGraph and replayed on fresh batches: every reply
    right.  World 1 with the process group up; the all-to-all is a device copy
    (tune sx_self_copy) because RCCL collectives issued on the engine's own
    comm stream crash graph instantiation on this ROCm stack (see
    tools/rccl_capture_probe.py -- torch's own captured all_to_all works)."""
    from conftest import free_port

    env = dict(os.environ, PTYPE_ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()),
               PTYPE_TUNE="sx_self_copy=1")
    try:
        r = subprocess.run([sys.executable, "-X", "faulthandler", "-c", _GRAPH_SCRIPT], env=env, capture_output=True, text=True,
                           timeout=120)
    except subprocess.TimeoutExpired as e:
        raise AssertionError("graph capture / replay hung; stderr: " + str(e.stderr)[-2000:]) from e
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    out = json.loads(line[0][7:])
    assert all(out["ok"]) and out["engine"] == "sorted" and out["agreed"], out


def test_alternate_sort_kernels_exact_in_a_subprocess():
    """The non-default sort kernels, switched by environment (read once per
    process): the sorted exchange's one-pass look-back sort (tune sx_sort=1) at
    R = 4, and the mailbox's count + scatter (mbox_sort=2) with the message-order
    drain (mbox_drain_msg=1) -- replies exact, unknown actors answered
    STATUS_NO_ACTOR."""
    code = textwrap.dedent("""
        import sys, threading, torch
        sys.path.insert(0, sys.argv[1])
        sys.path.insert(0, sys.argv[1] + "/tests")
        from test_sorted_exchange_gpu import _run_ranks, _table
        from ptype_amd.ops import batch as B
        from ptype_amd.ops.mailbox import Mailboxes
        from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, STATUS_OK
        from ptype_amd.parallel.exchange import ActorExchange
        R, n, M = 4, 8192, 120_000
        def body(r, fc, start, s):
            tab, _ = _table(n, R)
            st = torch.zeros(n // R + 1, dtype=torch.int64, device="cuda")
            ex = ActorExchange(tab, M, chunks=2, state=st, fake=(fc, r), delivery="mailbox", mailbox_ordered=False)
            start.wait()
            for k in range(4):
                req = B.gen_requests(M - 911 * r, n, METHOD_CALC_MULTIPLY, seed=70 + 5 * r + k, device="cuda")
                v, sts = ex.send(req)
                s.synchronize()
                assert bool((sts == STATUS_OK).all()) and torch.equal(v, req.a0 * req.a1), (r, k)
            assert ex.stats().failed == 0
            return True
        assert all(_run_ranks(R, body))
        tab, _ = _table(n, 1)
        mb = Mailboxes("cuda", shards=64, slots=1 << 12)
        from ptype_amd.ops.records import STATUS_NO_ACTOR
        for k in range(3):  # rings smaller than the traffic (~4.7 K messages per shard): the tail spills
            req = B.gen_requests(300_000, n + 64, METHOD_CALC_MULTIPLY, seed=9 + k, device="cuda")  # ids >= n: none
            v, sts = mb.send(req, tab, None)
            torch.cuda.synchronize()
            known = req.actor < n
            assert bool((sts[known] == STATUS_OK).all()) and torch.equal(v[known], (req.a0 * req.a1)[known]), k
            assert bool((sts[~known] == STATUS_NO_ACTOR).all()), k
        s = mb.stats()
        assert s["spilled"] > 0 and s["lookback_timeouts"] == 0
        print("SUBPROCESS-OK")
    """)
    env = dict(os.environ, PTYPE_TUNE="sx_sort=1,mbox_sort=2,mbox_drain_msg=1")
    p = subprocess.run([sys.executable, "-c", code, ROOT], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0 and "SUBPROCESS-OK" in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])


@pytest.mark.parametrize("M", [600_000, 4_500_000])
def test_sorted_exchange_loopback_both_tile_sizes_exact(M):
    """The sender's one-pass sort takes 1024-message tiles for a chunk of under 512
    4096-message tiles and 4096-message tiles above (exchange_sorted.hip): both
    exact on the loopback R = 8 pipeline (the bench's --loopback stand-in), Send
    after Send with new batches in the same tensors -- 600 K messages also run their
    collectives on the caller's stream (a small Send), 4.5 M on the comm stream."""
    R = 8
    n = 4096 * R
    tab, _ = _table(n, R)
    ex = ActorExchange(tab, M, chunks=2, state=torch.zeros(n // R + 1, dtype=torch.int64, device="cuda"),
                       fake=(hip().FakeComm(R, loopback=True), 0), delivery="mailbox", mailbox_ordered=False)
    req = B.MsgBatch(torch.empty(M, dtype=torch.int32, device="cuda"), torch.empty(M, dtype=torch.int64, device="cuda"),
                     torch.empty(M, dtype=torch.int64, device="cuda"), None, METHOD_CALC_MULTIPLY)
    val = torch.empty(M, dtype=torch.int64, device="cuda")
    st = torch.empty(M, dtype=torch.int32, device="cuda")
    for s in range(5):
        B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=40 + s, device="cuda", out=req)
        ex.send_all(req, out=(val, st))
        torch.cuda.synchronize()
        assert bool((st == STATUS_OK).all()) and torch.equal(val, req.a0 * req.a1), s
    assert ex.last_wire["S"] == 2 and ex.last_wire["agreed"]
    assert ex.stats().failed == 0

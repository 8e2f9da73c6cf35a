"""Wire format v3 (csrc/hip/packed.hpp): width-adaptive packed epoch records.

CPU tests pin the layout / reply-width rule (native vs the Python reference, and
the bounds themselves against brute force).  GPU tests compare every v3 kernel
with the CPU reference bit for bit: the v3 request regions are the v2 CPU
route's regions re-encoded, the v3 replies the v2 CPU dispatch's replies
re-encoded, and a multi-rank exchange simulated in one process (regions moved
between per-rank buffers the way the all-to-all moves them) returns exactly the
CPU reference pipeline's values and statuses.  The RCCL path of the native
engine (agreement all-reduce + packed all-to-alls) runs at world 1 in a child
process.
"""
import json
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest
import torch

from ptype_amd.ops import batch as B
from ptype_amd.ops import hip
from ptype_amd.ops import packed as P
from ptype_amd.ops.records import (METHOD_CALC_MULTIPLY, METHOD_ECHO, METHOD_PRIME_CHECK, STATUS_NO_ACTOR,
                                   STATUS_OK)
from ptype_amd.ops.table import RegistryTable, actor_keys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ----------------------------------------------------------------- CPU
def _rand_meta(rng):
    m = [0] * P.META_WORDS
    big = lambda: int(rng.integers(0, 2**64 - 1, dtype=np.uint64))  # noqa: E731
    for k in (P.META_MBOX, P.META_ARG0, P.META_ARG0 + 1, P.META_ARG0 + 2):
        m[k] = [0, 1, int(rng.integers(0, 2**16)), int(rng.integers(0, 2**40)), big(), 2**64 - 1][rng.integers(0, 6)]
    m[P.META_MBOX] = min(m[P.META_MBOX], (1 << 24) - 1)
    m[P.META_METHOD] = int(rng.integers(0, 9))
    m[P.META_MCOL] = int(rng.integers(0, 2))
    for f in range(8):
        m[P.META_FLAGS + f] = int(rng.integers(0, 2))
    return m


def test_layout_native_matches_reference():
    rng = np.random.default_rng(1)
    for _ in range(500):
        m = _rand_meta(rng)
        assert hip().packed_layout(m) == P.layout_reference(m), m
        assert hip().packed_reply_bits(m) == P.reply_bits_reference(m)
        assert hip().packed_req_words(1000, P.layout_reference(m)["S"]) == P.req_words(1000, P.layout_reference(m)["S"])


def test_headline_calculator_layout():
    """The bench's Calculator.Multiply traffic: 8-B requests, 4-B replies (v2: 20 + 9)."""
    g = torch.Generator().manual_seed(0)
    M = 100_000
    a = torch.randint(-2**15, 2**15, (M,), generator=g)
    b = torch.randint(0, 2**16, (M,), generator=g)
    actor = torch.randint(0, 8 * 131072, (M,), generator=g).to(torch.int32)
    a[0], b[0], actor[0] = -2**15, 2**16 - 1, 8 * 131072 - 1  # the extremes are in the batch
    m = P.meta_reference(B.MsgBatch(actor, a, b, None, METHOD_CALC_MULTIPLY), n_dir=8 * 131072, affine_w=8)
    L = P.layout_reference(m)
    assert L["w"] == [0, 17, 16, 17, 0] and L["S"] == 2 and L["vb"] == 4
    # the extreme product must round-trip through a 4-byte zigzag value
    p = np.int64(-2**15) * np.int64(2**16 - 1)
    assert int(P.zz(np.array([p]))[0]) < 2**32


def test_reply_bounds_cover_extremes():
    """For random column maxima, every reply a stateless handler can produce from
    arguments within the maxima fits the value plane."""
    rng = np.random.default_rng(7)
    for _ in range(300):
        wa, wb, wc = (int(rng.integers(0, 64)) for _ in range(3))
        za, zb, zc = (int(rng.integers(0, 2**w, dtype=np.uint64)) if w else 0 for w in (wa, wb, wc))
        m = [0] * P.META_WORDS
        m[P.META_ARG0:P.META_ARG0 + 3] = [za, zb, zc]
        for meth in (METHOD_CALC_MULTIPLY, METHOD_ECHO, METHOD_PRIME_CHECK):
            mm = list(m)
            mm[P.META_FLAGS + meth] = 1
            vb = P.layout_reference(mm)["vb"]
            # extreme arguments within the bounds: both signs at the largest magnitude
            ext = lambda z: [int(P.unzz(np.array([z], dtype=np.uint64))[0]),  # noqa: E731
                             int(P.unzz(np.array([max(z - 1, 0)], dtype=np.uint64))[0])]
            for x in ext(za):
                for y in ext(zb):
                    for t in ext(zc):
                        if meth == METHOD_CALC_MULTIPLY:
                            v = np.int64(x) * np.int64(y) if abs(x * y) < 2**63 else None
                        elif meth == METHOD_ECHO:
                            v = np.int64(x)
                        else:
                            v = np.int64(max(abs(x), abs(y), abs(t)) * (1 if t >= 0 else -1))
                        if v is None or vb == 8:
                            continue
                        assert int(P.zz(np.array([v]))[0]) < 2**(8 * vb), (meth, x, y, t, vb)


def test_pack_reference_roundtrip():
    rng = np.random.default_rng(3)
    for _ in range(50):
        m = _rand_meta(rng)
        L = P.layout_reference(m)
        if L["S"] > 8:
            continue
        n = 64
        fields = []
        for q in range(5):
            w = L["w"][q]
            hi = 2**w if w < 64 else 2**64
            fields.append(np.array([int(rng.integers(0, 2**62)) * 4 % hi if w else 0 for _ in range(n)], dtype=np.uint64))
        rec = P.pack_reference(fields, L)
        for q in range(5):
            w, off = L["w"][q], L["off"][q]
            if not w:
                continue
            words = [int.from_bytes(r.astype("<u4").tobytes(), "little") for r in rec]
            got = [(x >> off) & ((1 << w) - 1) for x in words]
            assert got == [int(v) for v in fields[q]]


# ----------------------------------------------------------------- GPU
def _tables(n, R, affine):
    g = RegistryTable(2 * n, device="cuda")
    c = RegistryTable(2 * n, device="cpu")
    ids = torch.arange(n)
    for t in (g, c):
        t.upsert(actor_keys(ids), (ids % R).to(torch.int32), (ids // R).to(torch.int32))
    if affine:
        g.enable_directory(n, affine_world=R)
    return g, c


def _mixed_batch(M, n, seed, mcol=True, big=False, nargs=3):
    gen = torch.Generator().manual_seed(seed)
    actor = torch.randint(0, n + 50, (M,), generator=gen).to(torch.int32)  # some unknown actors
    lim = 2**62 if big else 5000
    args = [torch.randint(-lim, lim, (M,), generator=gen) for _ in range(nargs)]
    args += [None] * (3 - nargs)
    if mcol:
        meth = torch.tensor([METHOD_CALC_MULTIPLY, METHOD_ECHO, METHOD_PRIME_CHECK])[torch.randint(0, 3, (M,), generator=gen)]
        if nargs == 3:  # Prime.Check over small ranges (its loop is per candidate)
            pc = meth == METHOD_PRIME_CHECK
            args[0] = torch.where(pc, args[0].abs() % 1000, args[0])
            args[1] = torch.where(pc, args[0] + 7, args[1])
        method = meth.to(torch.int16)
    else:
        method = METHOD_CALC_MULTIPLY
    return B.MsgBatch(actor, args[0], args[1], args[2], method)


def _cuda(b):
    t = lambda x: None if x is None else x.cuda()  # noqa: E731
    return B.MsgBatch(b.actor.cuda(), b.a0.cuda(), t(b.a1), t(b.a2), b.method if isinstance(b.method, int) else b.method.cuda())


@pytest.mark.gpu
@pytest.mark.parametrize("affine,mcol,big,nargs", [(True, False, False, 2), (False, True, False, 3),
                                                   (True, True, True, 3), (True, False, False, 1)])
def test_gpu_packed_meta_matches_reference(affine, mcol, big, nargs):
    n, M = 3000, 70_001
    g, _ = _tables(n, 4, affine)
    cb = _mixed_batch(M, n, 11, mcol=mcol, big=big, nargs=nargs)
    got = P.meta_list(P.meta(_cuda(cb), g))
    _, n_dir, aw = g.directory()
    assert got == P.meta_reference(cb, n_dir, aw, nargs)


@pytest.mark.gpu
@pytest.mark.parametrize("R,mcol,big,affine", [(1, False, False, True), (3, True, False, False),
                                               (8, True, True, True), (8, False, False, True)])
def test_gpu_packed_route_is_reencoded_v2(R, mcol, big, affine):
    n, M = 4000, 150_007
    C = B.stripe_capacity(M, R)
    g, c = _tables(n, R, affine)
    cb = _mixed_batch(M, n, R, mcol=mcol, big=big)
    gb = _cuda(cb)
    _, n_dir, aw = g.directory()
    L = P.layout(P.meta_reference(cb, n_dir, aw))
    send, perm, stats = P.route(gb, g, R, C, L, rank_self=0)
    fmt = B.FULL_FORMAT
    rsend, rperm, rstats = B.route(cb, c, R, C, rank_self=0, fmt=fmt)
    torch.cuda.synchronize()
    assert torch.equal(perm.cpu(), rperm)
    assert stats.cpu().tolist()[:2] == rstats.tolist()[:2]
    ref = P.requests_from_v2(rsend, R, C, fmt, L)
    W = P.req_words(C, L["S"])
    buf = send.cpu().numpy().view(np.uint32)
    for d, (h, recs) in enumerate(ref):
        reg = buf[d * W:(d + 1) * W]
        assert np.array_equal(reg[:4], h), d
        assert np.array_equal(reg[4:4 + recs.size].reshape(recs.shape), recs), d


def _simulate(batches, tables, states, R, C, L, packed, direct=False):
    """One exchange over R ranks in one process: route every rank, move the
    regions the way the all-to-all does, dispatch every rank, move the replies
    back, complete.  Returns per-rank (value, status) on the CPU."""
    dev = tables[0].device
    W = P.req_words(C, L["S"]) if packed else B.FULL_FORMAT.req_words(C)
    Wr = P.rep_words(C, L["vb"]) if packed else B.WireFormat.rep_words(C)
    sends, perms, outs = [], [], []
    for r in range(R):
        M = batches[r].M
        out = (torch.empty(M, dtype=torch.int64, device=dev), torch.empty(M, dtype=torch.int32, device=dev),
               torch.empty(max(C, 1), dtype=torch.int32, device=dev))
        dv = out if direct else None
        if packed:
            s, p, _ = P.route(batches[r], tables[r], R, C, L, rank_self=r, direct=dv)
        else:
            s, p, _ = B.route(batches[r], tables[r], R, C, rank_self=r, fmt=B.FULL_FORMAT, direct=dv)
        sends.append(s)
        perms.append(p)
        outs.append(out)
    replies = []
    for d in range(R):
        recv = torch.cat([sends[r][d * W:(d + 1) * W] for r in range(R)])
        dv = outs[d] if direct else None
        if packed:
            replies.append(P.dispatch(recv, R, C, L, state=states[d], direct=dv, rank_self=d))
        else:
            replies.append(B.dispatch(recv, R, C, states[d], fmt=B.FULL_FORMAT, direct=dv, rank_self=d))
    res = []
    for r in range(R):
        back = torch.cat([replies[d][r * Wr:(r + 1) * Wr] for d in range(R)])
        if packed:
            v, s = P.complete(back, perms[r], C, L["vb"], direct=direct, out_val=outs[r][0], out_status=outs[r][1])
        else:
            v, s = B.complete(back, perms[r], C, out_val=outs[r][0], out_status=outs[r][1], direct=direct)
        res.append((v.cpu(), s.cpu()))
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("R,mcol,big,direct", [(2, False, False, False), (3, True, False, True),
                                               (8, True, True, False), (8, False, False, True)])
def test_gpu_packed_exchange_simulated_ranks(R, mcol, big, direct):
    n, M = 2000, 40_000
    C = B.stripe_capacity(M, R)
    tabs = [_tables(n, R, True) for _ in range(R)]
    cbs = [_mixed_batch(M - 1000 * r, n, 100 + r, mcol=mcol and r != 1, big=big) for r in range(R)]  # rank 1: uniform
    metas = []
    for r in range(R):
        _, n_dir, aw = tabs[r][0].directory()
        metas.append(P.meta_list(P.meta(_cuda(cbs[r]), tabs[r][0])))
        assert metas[-1] == P.meta_reference(cbs[r], n_dir, aw)
    L = P.layout(P.combine(metas))
    gst = [torch.zeros(n // R + 1, dtype=torch.int64, device="cuda") for _ in range(R)]
    cst = [torch.zeros(n // R + 1, dtype=torch.int64) for _ in range(R)]
    got = _simulate([_cuda(b) for b in cbs], [t[0] for t in tabs], gst, R, C, L, packed=True, direct=direct)
    ref = _simulate(cbs, [t[1] for t in tabs], cst, R, C, L, packed=False, direct=direct)
    for r in range(R):
        assert torch.equal(got[r][1], ref[r][1]), r
        assert torch.equal(got[r][0], ref[r][0]), r
        assert int((got[r][1] == STATUS_NO_ACTOR).sum()) > 0
        assert int((got[r][1] == STATUS_OK).sum()) > M // 2


_ENGINE_SCRIPT = textwrap.dedent("""
    import json, os, sys, torch, torch.distributed as dist
    sys.path.insert(0, os.environ["PTYPE_ROOT"])
    from ptype_amd.ops import batch as B
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_ECHO, METHOD_COUNTER_ADD
    from ptype_amd.ops.table import RegistryTable, actor_keys
    from ptype_amd.parallel.exchange import ActorExchange
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from ptype_amd.parallel.native_group import solo_group
    G = solo_group(dev)  # the compiled DataPlane's RCCL communicator, world 1 (collectives forced on)
    n, M = 4096, 300_000
    g = RegistryTable(2 * n, device=dev)
    ids = torch.arange(n)
    g.upsert(actor_keys(ids), torch.zeros(n, dtype=torch.int32), ids.to(torch.int32))
    g.enable_directory(n, affine_world=1)
    gen = torch.Generator().manual_seed(3)
    cases = {
        "calc": B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=5, device=dev),
        "calc_unknown": B.gen_requests(M, n + 10, METHOD_CALC_MULTIPLY, seed=6, device=dev),
        "mixed_big": B.MsgBatch(torch.randint(0, n, (M,), generator=gen).to(torch.int32).to(dev),
                                torch.randint(-2**62, 2**62, (M,), generator=gen).to(dev),
                                torch.randint(-2**31, 2**31, (M,), generator=gen).to(dev), None,
                                torch.tensor([METHOD_CALC_MULTIPLY, METHOD_ECHO])[
                                    torch.randint(0, 2, (M,), generator=gen)].to(torch.int16).to(dev)),
        "counter": B.MsgBatch(torch.randint(0, n, (M,), generator=gen).to(torch.int32).to(dev),
                              torch.ones(M, dtype=torch.int64, device=dev), None, None, METHOD_COUNTER_ADD),
    }
    out = {}
    for name, req in cases.items():
        res = {}
        for packed in (True, False):
            st = torch.zeros(n, dtype=torch.int64, device=dev)
            ex = ActorExchange(g, M, chunks=3, state=st, packed=packed, group=G)
            assert ex.force_collectives
            ex.use_engine = packed  # v3 on the native engine vs the v2 Python pipeline
            v, s = ex.send(req)
            v2, s2 = ex.send(req)
            torch.cuda.synchronize()
            res[packed] = (v.cpu(), s.cpu(), v2.cpu(), s2.cpu(), st.cpu(), ex.last_wire, ex.stats().toowide)
        a, b = res[True], res[False]
        det = name != "counter"  # CounterAdd replies depend on the atomic order; the state does not
        same = all(torch.equal(x, y) for x, y in zip(a[:5] if det else (a[1], a[3], a[4]), b[:5] if det else (b[1], b[3], b[4])))
        if not det:
            same = same and int(a[0].sum()) == int(b[0].sum())
        out[name] = {"same": bool(same), "S": a[5]["S"], "vb": a[5]["vb"], "toowide": a[6],
                     "req_words": a[5]["req_words"], "rep_words": a[5]["rep_words"], "exact": a[5]["exact"]}
    print("RESULT " + json.dumps(out))
    G.close()
""")


@pytest.mark.gpu
@pytest.mark.parametrize("adaptive", ["1", "force"])
def test_gpu_engine_packed_rccl_world1(adaptive):
    """The native engine with wire v3 over RCCL (agreement all-reduce, packed
    all-to-alls) matches the v2 Python pipeline exactly, and sizes records as
    packed.hpp says (calculator: 2 dwords + 4-B replies).  ``force``: adaptive
    capacity at world 1, so the exact-size exchange runs on real RCCL -- the
    counts all-to-all and the grouped ncclSend / ncclRecv (to self)."""
    env = dict(os.environ, PTYPE_ROOT=ROOT, MASTER_ADDR="127.0.0.1",
               MASTER_PORT="29563" if adaptive == "1" else "29564", PTYPE_TUNE="adaptive_c=" + ("2" if adaptive == "force" else "1"))
    r = subprocess.run([sys.executable, "-c", _ENGINE_SCRIPT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
    assert line, r.stdout + r.stderr[-2000:]
    out = json.loads(line[0][7:])
    for name, o in out.items():
        assert o["same"], (name, o)
        assert o["toowide"] == 0, (name, o)
    assert out["calc"]["S"] == 2 and out["calc"]["vb"] == 4, out["calc"]
    assert out["calc_unknown"]["S"] == 2 and out["calc_unknown"]["vb"] == 4  # 24-bit mailbox field still fits
    assert out["mixed_big"]["vb"] == 8 and out["counter"]["vb"] == 8
    assert all(o["exact"] == (adaptive == "force") for o in out.values()), out

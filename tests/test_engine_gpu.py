"""Native epoch engine (csrc/hip/engine.hpp) vs the Python chunk pipeline:
same kernels, same schedule, so every output, state update and device counter
must be identical -- with and without RCCL collectives."""
import os
import subprocess
import sys
import textwrap

import pytest
import torch

from ptype_amd.ops import batch as B
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD, METHOD_ECHO, STATUS_NO_ACTOR
from ptype_amd.ops.table import RegistryTable, actor_keys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _table(n, affine):
    g = RegistryTable(2 * n, device="cuda")
    ids = torch.arange(n)
    g.upsert(actor_keys(ids), torch.zeros(n, dtype=torch.int32), ids.to(torch.int32))
    g.enable_directory(n, affine_world=1 if affine else 0)
    return g


@pytest.mark.gpu
@pytest.mark.parametrize("local", ["1", "0"])
@pytest.mark.parametrize("chunks,affine,mixed", [(1, True, False), (3, True, True), (4, False, True)])
def test_gpu_engine_matches_python_pipeline(chunks, affine, mixed, local, monkeypatch):
    """local=1: the engine's fused world-1 Send (local_send_kernel); local=0: its
    epoch-slot pipeline -- both against the Python slot pipeline."""
    from ptype_amd.parallel.exchange import ActorExchange

    monkeypatch.setenv("PTYPE_TUNE", f"local={local}")  # read when the engine is built

    n, M = 3000, 250_001
    gen = torch.Generator().manual_seed(chunks)
    actors = torch.randint(0, n + 40, (M,), generator=gen).to(torch.int32)  # some unknown ids
    method = (torch.randint(0, 3, (M,), generator=gen) if mixed else torch.zeros(M, dtype=torch.int64))
    method = torch.tensor([METHOD_ECHO, METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD])[method]
    a0 = torch.randint(-1000, 1000, (M,), generator=gen)
    a1 = torch.randint(-1000, 1000, (M,), generator=gen)
    a0 = torch.where(method == METHOD_COUNTER_ADD, torch.ones_like(a0), a0)  # +1 steps: order-free reply sums
    req = B.MsgBatch(actors.cuda(), a0.cuda(), a1.cuda(), None,
                     method.to(torch.int16).cuda() if mixed else METHOD_CALC_MULTIPLY)
    outs = {}
    for engine in (True, False):
        g = _table(n, affine)
        state = torch.zeros(n, dtype=torch.int64, device="cuda")
        ex = ActorExchange(g, M, chunks=chunks, state=state)
        ex.use_engine = engine
        ex.checksum = torch.zeros(1, dtype=torch.int64, device="cuda")
        val, st = ex.send(req)
        val2, st2 = ex.send(req)  # second step over reused buffers
        torch.cuda.synchronize()
        outs[engine] = (val.cpu(), st.cpu(), val2.cpu(), st2.cpu(), state.cpu(), ex.checksum.cpu(),
                        ex.stats().nomatch)
        assert (ex._engine is not None) == engine
        # the block-reduced checksum is the sum of every reply value returned
        total = int(val.sum()) + int(val2.sum())
        assert int(ex.checksum.item()) == total, (engine, int(ex.checksum.item()), total)
    # CounterAdd replies depend on the (atomic) order within a step; their sum,
    # the final state and everything else are deterministic
    det = method != METHOD_COUNTER_ADD
    for k, (a, b) in enumerate(zip(outs[True], outs[False])):
        if k in (0, 2):
            a, b = a[det], b[det]
        assert (a == b) if isinstance(a, int) else torch.equal(a, b), k
    assert int((outs[True][1] == STATUS_NO_ACTOR).sum()) > 0


_DIST_SCRIPT = textwrap.dedent("""
    import json, os, sys, torch, torch.distributed as dist
    sys.path.insert(0, os.environ["PTYPE_ROOT"])
    from ptype_amd.ops import batch as B
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY
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
    req = B.gen_requests(M, n + 10, METHOD_CALC_MULTIPLY, seed=5, device=dev)
    res = {}
    for engine in (True, False):
        ex = ActorExchange(g, M, chunks=3, group=G)
        assert ex.force_collectives
        ex.use_engine = engine
        v, s = ex.send(req)
        torch.cuda.synchronize()
        res[engine] = (v.cpu(), s.cpu(), ex._engine is not None)
    ok = torch.equal(res[True][0], res[False][0]) and torch.equal(res[True][1], res[False][1])
    print(json.dumps({"identical": bool(ok), "engine_used": res[True][2], "python_used": not res[False][2]}))
    G.close()
""")


@pytest.mark.gpu
def test_gpu_engine_rccl_world1_matches_python():
    """RCCL forced on at world 1: the engine's ncclAllToAll on the process
    group's communicator gives the same results as torch's all_to_all_single."""
    env = dict(os.environ, PTYPE_ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT="29561")
    r = subprocess.run([sys.executable, "-c", _DIST_SCRIPT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert '"identical": true, "engine_used": true, "python_used": true' in r.stdout, r.stdout + r.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("chunks,mixed", [(1, False), (2, True), (4, False)])
def test_gpu_engine_zero_copy_identity(chunks, mixed):
    """World 1, every actor known: the engine's fused local Send resolves and
    dispatches each message straight from the caller's columns (no epoch slot).
    Outputs and actor state equal the slot-copying Python pipeline's."""
    from ptype_amd.parallel.exchange import ActorExchange

    n, M = 5000, 300_007
    gen = torch.Generator().manual_seed(40 + chunks)
    actors = torch.randint(0, n, (M,), generator=gen).to(torch.int32)
    if mixed:
        method = torch.tensor([METHOD_ECHO, METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD])[torch.randint(0, 3, (M,), generator=gen)]
    else:
        method = torch.full((M,), METHOD_CALC_MULTIPLY)
    a0 = torch.randint(-10**6, 10**6, (M,), generator=gen)
    a0 = torch.where(method == METHOD_COUNTER_ADD, torch.ones_like(a0), a0)
    a1 = torch.randint(-10**6, 10**6, (M,), generator=gen)
    req = B.MsgBatch(actors.cuda(), a0.cuda(), a1.cuda(), None,
                     method.to(torch.int16).cuda() if mixed else METHOD_CALC_MULTIPLY)
    outs = {}
    for engine in (True, False):
        g = _table(n, True)
        state = torch.zeros(n, dtype=torch.int64, device="cuda")
        ex = ActorExchange(g, M, chunks=chunks, state=state)
        ex.use_engine = engine
        val, st = ex.send(req)
        torch.cuda.synchronize()
        outs[engine] = (val.cpu(), st.cpu(), state.cpu())
    det = method != METHOD_COUNTER_ADD
    assert torch.equal(outs[True][1], outs[False][1])
    assert torch.equal(outs[True][0][det], outs[False][0][det])
    assert int(outs[True][0][~det].sum()) == int(outs[False][0][~det].sum())
    assert torch.equal(outs[True][2], outs[False][2])
    assert bool((outs[True][1] == 0).all())

#!/usr/bin/env python3
"""The BASELINE.json configs other than the headline (bench.py), one JSON line each.

  host-rpc   example/calculator on the host path: control-plane member + net/rpc
             (HTTP CONNECT + gob over TCP) -- sync Call p50 RTT and concurrent
             Go throughput.  CPU only.
  gpu-1m     calculator actor, 1M synthetic messages per step, 1 MI355X
             (epoch slots in HBM + GPU registry), full Send path.
  optimus    optimus fan-out: Prime.Check ranges of many targets as one batch
             per step across every rank (torchrun for N GPUs: RCCL all-to-all
             dispatch), per-candidate delay 0.
  tell       device-side actor-to-actor messaging: token ring of Forward tells
             emitted by GPU handlers into the HBM outbox, pumped epoch by epoch.
  xproc      cross-process Call to a GPU actor on one node: shared-memory rings
             vs net/rpc over TCP (separate server and client processes).
  registry   1M-actor registry stress: GPU upsert / probe lookup / directory
             build / lease sweep / pack + snapshot to pinned host DRAM, and the
             control-plane store: puts with Raft snapshots + WAL.

usage: python tools/bench_suite.py {host-rpc,gpu-1m,optimus,registry} [...]
       torchrun --nproc-per-node N --master-addr 127.0.0.1 tools/bench_suite.py optimus
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def _emit(d):
    print(json.dumps(d), flush=True)


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# --------------------------------------------------------------------------- host-rpc
def host_rpc(a):
    from ptype_amd import cluster as C
    from ptype_amd.models.calculator import Args, Calculator

    os.environ.setdefault("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    pp, pc, sp = _free_port(), _free_port(), _free_port()
    d = tempfile.mkdtemp(prefix="hostrpc_")
    cfg = C.Config()
    cfg.service_name, cfg.node_name, cfg.port = "calculator", "n1", sp
    cfg.member = C.member_config(name="m0", dir=d, lpurls=[f"http://127.0.0.1:{pp}"],
                                 apurls=[f"http://127.0.0.1:{pp}"], lcurls=[f"http://127.0.0.1:{pc}"],
                                 acurls=[f"http://127.0.0.1:{pc}"], initial_cluster=f"m0=http://127.0.0.1:{pp}",
                                 unsafe_no_fsync=True)
    server = C.Serve(sp, Calculator(), host="127.0.0.1")
    c = C.Join(C.background(), cfg)
    try:
        for local in (False, True):
            client = c.NewClient("calculator", C.ConnConfig(allow_local=local, retries=0))
            for i in range(200):
                client.Call("Calculator.Multiply", Args(i, 3))
            lat = []
            for i in range(a.calls):
                t = time.perf_counter()
                client.Call("Calculator.Multiply", Args(i, 3))
                lat.append(time.perf_counter() - t)
            lat.sort()
            # throughput: many Go calls in flight from several threads
            n_threads, per = 8, a.calls // 2

            def worker(k):
                for i in range(per):
                    client.Call("Calculator.Multiply", Args(i, k))

            ths = [threading.Thread(target=worker, args=(k,)) for k in range(n_threads)]
            t0 = time.perf_counter()
            [t.start() for t in ths]
            [t.join() for t in ths]
            el = time.perf_counter() - t0
            _emit({"config": "example/calculator host path (net/rpc + gob over TCP)" if not local
                   else "example/calculator host path, in-process fast path (no socket)",
                   "p50_rtt_us": lat[len(lat) // 2] * 1e6, "p99_rtt_us": lat[int(len(lat) * 0.99)] * 1e6,
                   "msgs_per_s_8_threads": n_threads * per / el, "handler": "Python receiver (GIL)",
                   "device": "cpu"})
            client.Close()
    finally:
        c.Close()
        server.Close()


# --------------------------------------------------------------------------- gpu-1m
def gpu_1m(a):
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # 8 whole steps per graph replay: at 1 Mi messages the graph launch is a third of a step
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--msgs-per-gpu", str(a.msgs),
                        "--steps", str(8 * max(1, a.steps // 8)), "--warmup", "8", "--steps-per-graph", "8",
                        "--actors-per-gpu", str(a.actors)],
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-2000:])
    line = json.loads(r.stdout.strip().splitlines()[-1])
    line["config_name"] = "calculator actor, 1M synthetic msgs, 1 MI355X"
    _emit(line)


# --------------------------------------------------------------------------- optimus
def optimus(a):
    import torch.distributed as dist

    from ptype_amd.ops import batch as B
    from ptype_amd.ops.records import METHOD_PRIME_CHECK, STATUS_OK
    from ptype_amd.ops.table import RegistryTable, actor_keys
    from ptype_amd.parallel.exchange import ActorExchange

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    fake = None
    geo = world
    if a.loopback > 0:  # rank 0 of a symmetric R-rank node; all-to-alls as local copies (FakeComm)
        from ptype_amd.ops import hip

        fake = (hip().FakeComm(a.loopback, loopback=True, link_gbps=a.link_gbps), 0)
        geo = a.loopback
    per = a.actors
    n = per * geo
    table = RegistryTable(2 * n, device=dev)
    ids = torch.arange(n, dtype=torch.int64)
    table.upsert(actor_keys(ids), (ids % geo).to(torch.int32), (ids // geo).to(torch.int32))
    table.enable_directory(n, affine_world=geo)
    # targets: odd numbers around `base`, each split into 10-wide ranges [2,10), [10,20), ...
    T = a.targets
    tg = torch.arange(T, dtype=torch.int64, device=dev) * 2 + a.base + rank * 2 * T + 1
    nr = (tg + 9) // 10  # ranges per target (splitWork: i = 10, 20, ... < target + 10)
    M = int(nr.sum())
    tid = torch.repeat_interleave(torch.arange(T, device=dev), nr)
    first = torch.cumsum(nr, 0) - nr
    k = torch.arange(M, device=dev) - first[tid]
    lo = torch.where(k == 0, torch.full_like(k, 2), k * 10)
    hi = (k + 1) * 10
    batch = B.MsgBatch((torch.arange(M, device=dev) % n).to(torch.int32), lo, hi, tg[tid], METHOD_PRIME_CHECK)
    ex = ActorExchange(table, M, chunks=4 if geo > 1 else 1, fake=fake)
    tg_rep = tg[tid]

    def step():
        val, st = ex.send(batch)
        # gather: per target, the smallest reply that is not the target (watchReplies' winner
        # when all replies are in); target itself when it is prime
        # segmented min over each target's contiguous ranges (no contended atomics;
        # float64 is exact for these magnitudes)
        cand = torch.where(val != tg_rep, val, torch.full_like(val, 1 << 52)).double()
        best = torch.segment_reduce(cand, "min", lengths=nr).long()
        return torch.where(best == (1 << 52), tg, best), st

    for _ in range(3):
        ans, st = step()
    torch.cuda.synchronize()
    assert bool((st == STATUS_OK).all())
    # check against a CPU trial division on a sample
    for j in range(0, T, max(1, T // 64)):
        t = int(tg[j])
        exp = next((d for d in range(2, t) if t % d == 0), t)
        assert int(ans[j]) == exp, (t, int(ans[j]), exp)
    if world > 1:
        dist.barrier(device_ids=[local])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier(device_ids=[local])
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        extra = {}
        if fake is not None:
            extra = {"loopback_ranks": a.loopback, "link_gbps": a.link_gbps, "wire": (ex.last_wire or {}).get("S"),
                     "note": "profiling mode: rank 0 of a symmetric R-rank node, all-to-alls as local copies "
                             "(modelled link bandwidth if link_gbps > 0); per-GPU rates, not a node total"}
        _emit({**extra, "config": "example/optimus fan-out, RCCL all-to-all dispatch" if world > 1 else
               "example/optimus fan-out, %d-rank loopback on 1 GPU" % geo if fake else
               "example/optimus fan-out, 1 GPU", "n_gpus": world, "targets_per_gpu_per_step": T,
               "ranges_per_gpu_per_step": M, "ranges_per_s": M * world * a.steps / el,
               "targets_per_s": T * world * a.steps / el, "ms_per_step": el / a.steps * 1e3,
               "candidates_per_range": 10, "delay_per_candidate": 0})
    if world > 1:
        dist.destroy_process_group()


# --------------------------------------------------------------------------- tell
def tell(a):
    """Device-side actor-to-actor messaging: a token ring where every hop is a
    message emitted by a GPU handler into the HBM outbox and routed by the next
    exchange epoch (torchrun for N GPUs: hops cross GPUs over RCCL)."""
    import torch.distributed as dist

    from ptype_amd.ops import batch as B
    from ptype_amd.ops.outbox import DeviceOutbox
    from ptype_amd.ops.records import METHOD_FORWARD
    from ptype_amd.ops.table import RegistryTable, actor_keys
    from ptype_amd.parallel.exchange import ActorExchange

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    per, T, H = a.actors, a.tokens, a.hops
    n = per * world
    table = RegistryTable(2 * n, device=dev)
    ids = torch.arange(n, dtype=torch.int64)
    table.upsert(actor_keys(ids), (ids % world).to(torch.int32), (ids // world).to(torch.int32))
    table.enable_directory(n, affine_world=world)
    state = torch.zeros(per, dtype=torch.int64, device=dev)
    ex = ActorExchange(table, T, chunks=1, state=state)
    outbox = DeviceOutbox(T, device=dev)
    stride = 7919
    starts = (torch.arange(T, dtype=torch.int64, device=dev) * 97 + rank * 13) % n
    init = B.MsgBatch(starts.to(torch.int32), (starts + stride) % n, torch.full((T,), H, dtype=torch.int64, device=dev),
                      torch.full((T,), stride | (n << 32), dtype=torch.int64, device=dev), METHOD_FORWARD)
    ex.pump(outbox, initial=init.slice(0, min(T, 1024)))  # warm-up
    state.zero_()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier(device_ids=[local])
    t0 = time.perf_counter()
    epochs, delivered = ex.pump(outbox, initial=init)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tot = torch.tensor([delivered, int(state.sum())], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(tot)
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    assert int(tot[1]) == T * world * (H + 1) and outbox.dropped == 0, (tot.tolist(), outbox.dropped)
    if rank == 0:
        _emit({"config": "device-side actor messaging (token ring, Forward tells via HBM outbox)", "n_gpus": world,
               "tokens_per_gpu": T, "hops": H, "epochs": epochs, "messages": int(tot[0]),
               "messages_per_s": int(tot[0]) / el, "ms_per_epoch": el / max(epochs, 1) * 1e3})
    if world > 1:
        dist.destroy_process_group()


# --------------------------------------------------------------------------- xproc
def _xproc_server(port, q, stop):
    from ptype_amd import cluster as C
    from ptype_amd.models import calculator
    from ptype_amd.runtime import DeviceRuntime

    rt = DeviceRuntime(torch.device("cuda", 0), actors=1024, idle_ms=200.0)
    server = C.Server()
    calculator.serve_device(rt, server)
    server.Listen(port, "127.0.0.1")
    q.put(("ready", rt.server.shm_name))
    stop.wait(300)
    q.put(("server", {"ring_on_device": bool(rt.server.ring_on_device), "ring_fds_handed": rt.server.ring_fds_handed}))
    server.Close()
    rt.close()


def _pcts(lat):
    lat.sort()
    return {"p50_us": lat[len(lat) // 2] * 1e6, "p90_us": lat[int(len(lat) * 0.9)] * 1e6,
            "p99_us": lat[int(len(lat) * 0.99)] * 1e6}


def _xproc_client(port, seg, calls, q):
    os.environ["HIP_VISIBLE_DEVICES"] = ""  # the client process never touches a GPU
    from ptype_amd import _core
    from ptype_amd.models.calculator import Args
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY

    out = {}
    for name, allow in (("shm", True), ("tcp", False)):
        c = _core.dial_http("127.0.0.1", port, 5.0, allow)
        for i in range(500):
            c.call("Calculator.Multiply", Args(i, 2))
        lat = []
        for i in range(calls):
            t = time.perf_counter()
            c.call("Calculator.Multiply", Args(i, 3))
            lat.append(time.perf_counter() - t)
        out[name] = {"transport": c.transport, "ring": c.ring_placement, **_pcts(lat)}
        c.close()
    # the same ring without net/rpc's name lookup and gob argument encoding
    raw = _core.ShmClient(seg)
    lat = []
    for i in range(calls + 500):
        t = time.perf_counter()
        raw.call(METHOD_CALC_MULTIPLY, i % 1024, i, 3)
        if i >= 500:
            lat.append(time.perf_counter() - t)
    out["raw"] = {"ring": raw.ring_placement, **_pcts(lat)}
    q.put(("client", out))


def xproc(a):
    """example/calculator's shape with GPU actors: server and client are separate
    processes on one node; the client's Call reaches the GPU actor through the
    dispatcher's rings (request ring in the server GPU's memory, mapped from its
    dma-buf; replies in shared memory) vs net/rpc over TCP to the same server.
    `raw` is the same ring called without net/rpc's method lookup and gob args."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q, stop = ctx.Queue(), ctx.Event()
    port = _free_port()
    sp = ctx.Process(target=_xproc_server, args=(port, q, stop))
    sp.start()
    kind, seg = q.get(timeout=300)
    assert kind == "ready"
    cp = ctx.Process(target=_xproc_client, args=(port, seg, a.calls, q))
    cp.start()
    kind, out = q.get(timeout=300)
    assert kind == "client", out
    cp.join(30)
    stop.set()
    _, srv = q.get(timeout=60)
    sp.join(60)
    _emit({"config": "cross-process Call to a GPU actor on the same node (calculator server + client processes)",
           "request_ring": os.environ.get("PTYPE_XPROC_RING", "device"), "server": srv,
           "shm": out["shm"], "shm_raw": out["raw"], "tcp_netrpc": out["tcp"]})


# --------------------------------------------------------------------------- registry
def registry(a):
    from ptype_amd.ops import batch as B
    from ptype_amd.ops.table import RegistryTable, actor_keys

    dev = torch.device("cuda", 0)
    N = a.actors
    out = {"config": "1M-actor registry stress + snapshot to pinned host DRAM", "actors": N}

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / reps

    keys = actor_keys(torch.arange(N, dtype=torch.int64)).to(dev)
    ranks = (torch.arange(N, device=dev) % 8).to(torch.int32)
    mbox = (torch.arange(N, device=dev) // 8).to(torch.int32)
    exp = torch.full((N,), 1 << 40, dtype=torch.int64, device=dev)
    # inserts into an empty table (table allocation outside the timed region)
    ins = []
    for _ in range(5):
        t = RegistryTable(4 * N, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t.upsert(keys, ranks, mbox, exp)
        torch.cuda.synchronize()
        ins.append(time.perf_counter() - t0)
    out["insert_ops_per_s"] = N / min(ins)
    s = timed(lambda: t.upsert(keys, ranks, mbox, exp))  # every key present: in-place updates
    out["update_ops_per_s"] = N / s
    out["table_bytes"] = t.cap * 16
    q = keys[torch.randperm(N, device=dev)]
    s = timed(lambda: t.lookup(q))
    out["lookup_ops_per_s"] = N / s

    def build_dir():
        t._dir_dirty = True
        t.directory()

    t.enable_directory(N)
    s = timed(build_dir)
    out["directory_build_ms"] = s * 1e3
    s = timed(lambda: t.sweep(1))  # nothing expires: a full scan
    out["sweep_scan_ms"] = s * 1e3
    s = timed(lambda: t.pack())
    out["pack_ms"] = s * 1e3
    # K7 straight into pinned host DRAM; the pinned buffers are allocated by the
    # first snapshot of a table and reused (the first call is timed separately)
    side = torch.cuda.Stream(dev)
    t0 = time.perf_counter()
    h_ent, h_exp = t.snapshot_to_host(side)
    out["snapshot_first_ms_incl_pinned_alloc"] = (time.perf_counter() - t0) * 1e3
    els = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h_ent, h_exp = t.snapshot_to_host(side)
        els.append(time.perf_counter() - t0)
    el = min(els)
    nbytes = h_ent.numel() * 8 + h_exp.numel() * 8
    out["snapshot_to_pinned_ms"] = el * 1e3
    out["snapshot_to_pinned_ms_median"] = sorted(els)[len(els) // 2] * 1e3
    out["snapshot_bytes"] = nbytes
    out["snapshot_gb_per_s"] = nbytes / el / 1e9
    out["table_scanned_bytes"] = t.cap * 24
    rest = []
    for _ in range(3):
        t2 = RegistryTable(2 * N, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t2.load_packed(h_ent, h_exp)  # one H2D copy per array + one packed upsert kernel
        torch.cuda.synchronize()
        rest.append(time.perf_counter() - t0)
        assert t2.live == N
    out["restore_ms"] = min(rest) * 1e3
    out["restore_gb_per_s"] = nbytes / min(rest) / 1e9
    del B
    # control-plane store: puts through Raft with WAL + periodic snapshots
    from ptype_amd import cluster as C

    os.environ.setdefault("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    pp, pc = _free_port(), _free_port()
    d = tempfile.mkdtemp(prefix="regstress_")
    cfg = C.Config()
    cfg.service_name, cfg.node_name, cfg.port = "stress", "n1", _free_port()
    cfg.member = C.member_config(name="m0", dir=d, lpurls=[f"http://127.0.0.1:{pp}"],
                                 apurls=[f"http://127.0.0.1:{pp}"], lcurls=[f"http://127.0.0.1:{pc}"],
                                 acurls=[f"http://127.0.0.1:{pc}"], initial_cluster=f"m0=http://127.0.0.1:{pp}",
                                 snapshot_count=2000)
    c = C.Join(C.background(), cfg)
    try:
        n_puts = a.puts
        t0 = time.perf_counter()
        for i in range(n_puts):
            c.Store.Put(C.background(), f"actors/{i}", "x" * 32)
        el = time.perf_counter() - t0
        out["store_puts_per_s_fsync"] = n_puts / el
        # group commit: concurrent writers share one WAL fdatasync per raft-loop round
        import threading

        def writer(k):
            for i in range(n_puts // 8):
                c.Store.Put(C.background(), f"g{k}/{i}", "x" * 32)

        ths = [threading.Thread(target=writer, args=(k,)) for k in range(8)]
        t0 = time.perf_counter()
        [t.start() for t in ths]
        [t.join() for t in ths]
        out["store_puts_per_s_fsync_8_writers"] = 8 * (n_puts // 8) / (time.perf_counter() - t0)
        # linearizable reads: a ReadIndex round each, no log entry
        c0 = c._c.member_status().commit
        t0 = time.perf_counter()
        for i in range(n_puts):
            c.Store.Get(C.background(), f"actors/{i % 100}")
        out["store_linearizable_gets_per_s"] = n_puts / (time.perf_counter() - t0)
        out["store_log_entries_per_get"] = (c._c.member_status().commit - c0) / n_puts
        out["store_snapshot_on_disk"] = os.path.exists(os.path.join(d, "member", "snap.bin"))
    finally:
        c.Close()
    _emit(out)


# --------------------------------------------------------------------------- gob (K4)
def gob(a):
    """K4: gob value messages of calculator Args{A, B} for a batch in HBM --
    encode (size / scan / write passes) and decode (one message per lane)."""
    from ptype_amd.ops import batch as B
    from ptype_amd.ops import gob as G

    M = a.msgs
    req = B.gen_requests(M, 1 << 17, seed=5, device="cuda")
    cols = [req.a0.contiguous(), req.a1.contiguous()]
    buf, offs = G.encode_structs(cols, 65)
    back, st = G.decode_structs(buf, offs, 2, 65)
    torch.cuda.synchronize()
    assert not bool(st.any()) and torch.equal(back[0], cols[0]) and torch.equal(back[1], cols[1])

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps

    te = timed(lambda: G.encode_structs(cols, 65))
    td = timed(lambda: G.decode_structs(buf, offs, 2, 65))
    nbytes = int(buf.numel())
    _emit({"config": "K4 gob value messages, calculator Args{A, B}", "messages": M, "gob_bytes": nbytes,
           "bytes_per_message": nbytes / M, "encode_ms": te * 1e3, "encode_msgs_per_s": M / te,
           "decode_ms": td * 1e3, "decode_msgs_per_s": M / td, "decode_gob_GBps": nbytes / td / 1e9})


def main():
    p = argparse.ArgumentParser()
    p.add_argument("which", choices=["host-rpc", "gpu-1m", "optimus", "registry", "tell", "xproc", "gob"])
    p.add_argument("--calls", type=int, default=4000)
    p.add_argument("--msgs", type=int, default=1 << 20)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--actors", type=int, default=0)
    p.add_argument("--targets", type=int, default=8192)
    p.add_argument("--loopback", type=int, default=0, metavar="R", help="optimus: R-rank loopback (FakeComm)")
    p.add_argument("--link-gbps", type=float, default=0.0, help="optimus --loopback: modelled link bandwidth")
    p.add_argument("--base", type=int, default=100_001)
    p.add_argument("--puts", type=int, default=5000)
    p.add_argument("--tokens", type=int, default=1 << 20)
    p.add_argument("--hops", type=int, default=32)
    a = p.parse_args()
    if not a.actors:
        a.actors = {"registry": 1 << 20, "optimus": 65536}.get(a.which, 131072)
    {"host-rpc": host_rpc, "gpu-1m": gpu_1m, "optimus": optimus, "registry": registry, "tell": tell,
     "xproc": xproc, "gob": gob}[a.which](a)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Headline benchmark: messages/sec (whole node) + p50 RPC RTT, calculator actor.

BASELINE.json metric: "messages/sec (whole node) + p50 RPC RTT, calculator actor
at 1/2/4/8 MI355X".  One process per GPU (torchrun); every rank hosts a shard of
the calculator actors and is also a client that sends a batch of synthetic
``Calculator.Multiply(Args{A, B})`` calls (example/calculator/calculator.go:3-12)
to uniformly random actors across the whole node each step.

A timed step is the full `Send` path for the batch: generate the requests
(client), K1 GPU-registry lookup + bucket, RCCL all-to-all over xGMI, K3
dispatch through the handler table, RCCL all-to-all of replies, K8 completion
into message order.  Nothing is cached across steps (new args every step) and
the results of a step are verified against ``A * B``.

p50 RTT: single synchronous ``Call``s to a GPU actor through the persistent
dispatcher (host-visible ring, no launch per call), measured after the timed
loop on every rank's own GPU.

Placement: actors are spread over the ranks and their mailboxes by a random
permutation (``--placement random``, the default), so every message's route is
read from the GPU registry mirror (the compiled route directory; ``--lookup hash``
probes the hash table instead).  ``--placement affine`` (actor a on rank a % N,
mailbox a / N) lets the route be computed without registry reads; it is reported
as a secondary figure, never as the headline.

Usage: python bench.py [--gpus N --steps K --warmup W]
  N > 1 without torchrun: bench.py starts torch.distributed.run with N rank
  processes itself (a child process, before anything touches a GPU) and exits
  with its status.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import weakref


def _parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=8)
    p.add_argument("--msgs-per-gpu", type=int, default=8 * 1024 * 1024, help="messages each rank sends per step")
    p.add_argument("--actors-per-gpu", type=int, default=131072)
    p.add_argument("--chunks", type=int, default=0, help="pipeline chunks per step (0 = auto)")
    p.add_argument("--rtt-calls", type=int, default=2000)
    p.add_argument("--cpu", action="store_true", help="gloo/CPU dry run of the same pipeline (tests)")
    p.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                   help="replay the step as a captured hipGraph (auto: single rank)")
    p.add_argument("--steps-per-graph", type=int, default=0,
                   help="whole steps per graph replay (the graph launch and the seed advance show per replay); "
                        "steps and warmup must be multiples.  0 = auto: the largest of 4, 2, 1 dividing both")
    p.add_argument("--loopback", type=int, default=0, metavar="R",
                   help="profiling only: one GPU runs rank 0 of a symmetric R-rank node with the all-to-alls "
                        "as local copies (FakeComm loopback) -- the compute side of an R-GPU step")
    p.add_argument("--link-gbps", type=float, default=0.0,
                   help="with --loopback: model the all-to-all at this per-rank off-rank bandwidth (GB/s)")
    p.add_argument("--force-dist", action="store_true",
                   help="initialise the process group and run the all-to-alls even for one rank "
                        "(exercises the RCCL path on a 1-GPU box)")
    p.add_argument("--placement", choices=["random", "affine"], default="random",
                   help="actor -> (rank, mailbox) placement: a random permutation (routes read the registry) "
                        "or the strided rule (routes computed)")
    p.add_argument("--lookup", choices=["directory", "hash"], default="directory",
                   help="registry mirror read on the route: compiled route directory or hash-table probe")
    p.add_argument("--delivery", choices=["direct", "mailbox"], default="mailbox",
                   help="how a message reaches its actor on its GPU: through the HBM mailboxes (BASELINE config "
                        "2: K2 enqueue + K3 drain; at N > 1 on receipt), or one fused resolve-and-run pass")
    p.add_argument("--sharding", choices=["actor", "arrival"], default="actor",
                   help="mailbox rings: per actor (every actor's messages FIFO in one ring) or per arrival tile")
    p.add_argument("--mailbox-shards", type=int, default=256, help="HBM mailbox shard rings per GPU")
    p.add_argument("--mailbox-slots", type=int, default=0, help="slots per mailbox ring (0: 2x the uniform load)")
    p.add_argument("--zipf", type=float, default=0.0, metavar="S",
                   help="skewed load: actor popularity Zipf(S) (hot actors scattered over the GPUs); batches "
                        "pre-generated outside the timed loop, so compare against --zipf 0 --pregen")
    p.add_argument("--pregen", action="store_true", help="uniform load, pre-generated like --zipf (A/B baseline)")
    p.add_argument("--method", choices=["multiply", "seqfold"], default="multiply",
                   help="the timed step's method (seqfold: the ordered stateful method -- experiments; "
                        "the headline is Calculator.Multiply)")
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the secondary (affine placement) measurement after the headline")
    p.add_argument("--comm", choices=["rccl", "ipc"], default="rccl",
                   help="N > 1 data-plane transport of the compiled DataPlane (csrc/core/dataplane.cpp): RCCL over "
                        "xGMI (one GPU per rank), or IpcComm (csrc/hip/ipc_comm.hpp: shared-memory segments) -- ipc "
                        "lets every rank share one GPU: a multi-process rehearsal, not a scaling figure")
    return p.parse_args()


def _spawn_ranks(args) -> int:
    """`--gpus N` outside torchrun: run this script under torch.distributed.run with
    N local rank processes (127.0.0.1 rendezvous) as a child; return its status.
    Runs before anything initialises a GPU in this process (no exec)."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


_LIVE_EXCHANGES: list = []  # for the hang watchdog
_EMIT_ON_HANG: list = [None]  # rank 0's JSON line, printed by the watchdog if a last secondary hangs


def _hang_watchdog(after_s: float, rank: int) -> None:
    """Hang watchdog (PTYPE_HANG_DIAG=<seconds>; on by default with more than one
    rank, PTYPE_HANG_DIAG=0 turns it off): if the run has not finished after that
    long, print every engine's hand-off words (signalled sequence vs value the GPU
    wrote) and whether its streams drained, then exit 3 -- the main thread is
    blocked inside a synchronisation and cannot report, and a multi-GPU run that
    hangs should end with a diagnosis rather than at the launcher's time limit."""
    import threading

    import torch

    def dump():
        print(f"[rank {rank}] HANG after {after_s:.0f} s", file=sys.stderr, flush=True)
        if _EMIT_ON_HANG[0] is not None:  # only the last secondary is left: report the line, end cleanly
            try:
                _EMIT_ON_HANG[0]()
            finally:
                os._exit(0)
        names = ["routed", "req_in", "served", "rep_in"]
        for ref in _LIVE_EXCHANGES:
            ex = ref()
            eng = ex._engine if ex is not None else None
            if eng is None:
                continue
            st = eng.hang_state(torch.cuda.current_stream(ex.device).cuda_stream)
            for k in range(32):
                seq, val = st[2 * k], st[2 * k + 1]
                if seq or val > 0:
                    print(f"  {names[k // 8]}[buf {k % 8}]: signalled {seq}, GPU wrote {val}"
                          + ("   <-- behind" if val >= 0 and val < seq else ""), file=sys.stderr, flush=True)
            print(f"  compute stream drained: {bool(st[64])}, comm stream drained: {bool(st[65])}, "
                  f"layout agreement done: {bool(st[66])}, route kernels done per chunk: {st[67:75]}",
                  file=sys.stderr, flush=True)
        os._exit(3)

    t = threading.Timer(after_s, dump)
    t.daemon = True
    t.start()


def place_actors(n_actors: int, world: int, placement: str, seed: int = 1234):
    """(rank, mailbox) of every actor id: the same on every rank (CPU generator).
    random: a uniformly random bijection onto rank-major mailbox slots, so each
    rank hosts exactly n_actors / world mailboxes."""
    import torch

    ids = torch.arange(n_actors, dtype=torch.int64)
    if placement == "affine":
        slot = ids
    else:
        slot = torch.randperm(n_actors, generator=torch.Generator().manual_seed(seed))
    return (slot % world).to(torch.int32), (slot // world).to(torch.int32)


def wire_info(ex, req) -> dict:
    """Bytes per message on the all-to-alls: wire v3 (packed, agreed per Send) when
    the exchange ran collectives through the native engine, else wire v2."""
    from ptype_amd.ops import batch as B

    w = ex.last_wire
    if w is not None and w["S"]:
        # exact: the regions' used prefixes move (counts all-to-all + grouped send/recv);
        # padded: every peer region at the agreed capacity
        return {"wire": "v3-packed", "record_bytes": 4 * w["S"], "reply_bytes": w["vb"] + 0.125,
                "field_bits": w["w"], "exchange": "exact" if w.get("exact") else ("per-pair prefixes" if w.get("pairs") else "padded"),
                "engine": w.get("engine", "epoch"),
                "wire_bytes_per_msg": 4 * (w["req_words"] + w["rep_words"]) * ex.chunks / max(req.M, 1)}
    return {"wire": "v2", "record_bytes": 4 * (ex.fmt or B.WireFormat.for_batch(req)).stride, "reply_bytes": 9}


def main():
    args = _parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_spawn_ranks(args))
    import torch
    import torch.distributed as dist

    from ptype_amd.ops import batch as B
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_SEQ_FOLD, STATUS_OK
    from ptype_amd.ops.table import RegistryTable, actor_keys
    from ptype_amd.parallel.exchange import ActorExchange

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"--gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    use_gpu = not args.cpu
    ipc = use_gpu and args.comm == "ipc" and world > 1
    if use_gpu:
        dev_idx = local % max(1, torch.cuda.device_count()) if ipc else local  # ipc: ranks may share a GPU
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    dist_on = world > 1 or args.force_dist
    # N > 1 on GPUs: the data plane the way Join forms it -- a control-plane member per
    # rank and the compiled DataPlane's communicator (RCCL over xGMI, or IpcComm with
    # --comm ipc), no torch process group.  CPU runs: a gloo group.
    native = dist_on and use_gpu
    M = args.msgs_per_gpu
    chunks = args.chunks or (2 if dist_on or args.loopback else 1)
    G = bench_cp = None
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        if native:
            from ptype_amd.parallel.exchange import ipc_cap_for
            from ptype_amd.utils import benchmarks as BM

            # (IpcComm regions: as large as the largest exchange of the run -- the headline's,
            # or the optimus secondary's fan-out batch)
            cap = ipc_cap_for(M, chunks, world)
            if not args.no_secondary:
                cap = max(cap, ipc_cap_for(BM.optimus_max_batch(world), chunks, world))
            bench_cp, G = BM.bench_group(device, rank, world, comm="ipc" if ipc else "rccl",
                                         cap_bytes=cap if ipc else 0)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)

    def barrier():
        if dist_on:
            if native:
                G.barrier()
            else:
                dist.barrier()

    def max_over_ranks(x: float) -> float:
        if not dist_on:
            return x
        if native:
            return G.max_over_ranks(x)
        tt = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    def sync():
        if use_gpu:
            torch.cuda.synchronize(device)

    fake = None
    if args.loopback > 0:
        if world != 1 or not use_gpu:
            raise SystemExit("--loopback is a single-process GPU profiling mode")
        from ptype_amd.ops import hip

        fake = (hip().FakeComm(args.loopback, loopback=True, link_gbps=args.link_gbps), 0)
    geo = args.loopback or world  # ranks the actors are sharded over
    n_actors = args.actors_per_gpu * geo
    # (2 pipeline chunks on the collective path: measured against 1/4/8 with the
    # all-to-all modelled at xGMI-like bandwidth, profiles/r1_chunk_model.jsonl,
    # and on the forced single-rank RCCL path: 0.31 vs 0.38-0.40 ms at 4 chunks)

    def build_table(placement):
        # GPU registry mirror: every actor of the node -> (rank, mailbox)
        t = RegistryTable(2 * n_actors, device=device)
        ids = torch.arange(n_actors, dtype=torch.int64)
        r, mb = place_actors(n_actors, geo, placement)
        t.upsert(actor_keys(ids), r, mb)
        if args.lookup == "directory":
            # K5b route directory; the device verifies the strided rule (affine placement only)
            t.enable_directory(n_actors, affine_world=geo)
        return t

    state = torch.zeros(args.actors_per_gpu, dtype=torch.int64, device=device)
    req = B.MsgBatch(torch.empty(M, dtype=torch.int32, device=device), torch.empty(M, dtype=torch.int64, device=device),
                     torch.empty(M, dtype=torch.int64, device=device), None, METHOD_CALC_MULTIPLY)
    val = torch.empty(M, dtype=torch.int64, device=device)
    st = torch.empty(M, dtype=torch.int32, device=device)
    pregen = args.zipf > 0 or args.pregen
    use_graph = use_gpu and not pregen and (args.graph == "on" or (args.graph == "auto" and not dist_on and fake is None))
    if args.steps_per_graph == 0:  # auto (measured at 8 Mi msgs: 1 -> 89-90, 2 -> 93.8, 4 -> 94.8 G msg/s, round 2)
        # the timed steps replay a graph of U whole steps (U divides --steps); warm-up
        # steps that do not fill a U-step replay run on a 1-step graph of the same
        # step, so exactly --warmup steps warm up and exactly --steps are timed
        # (round 4: 20 steps per replay measured 1-3 % above 4 at 8 Mi and 1 Mi, profiles/r4_mailbox_ab.md)
        args.steps_per_graph = next((u for u in (20, 10, 5, 4, 2) if use_graph and args.steps % u == 0), 1)
    if args.steps_per_graph < 1 or (args.steps_per_graph > 1 and (
            not use_graph or args.steps % args.steps_per_graph)):
        raise SystemExit("--steps-per-graph: needs the graph path, and --steps a multiple of it")
    pre = []
    if pregen:  # 4 distinct batches per rank, generated before any timing
        for k in range(4):
            sd = (k * world + rank) * 7919 + 13
            pre.append(B.gen_zipf_requests(M, n_actors, args.zipf, seed=sd, device=device) if args.zipf > 0 else
                       B.gen_requests(M, n_actors, METHOD_CALC_MULTIPLY, seed=sd, device=device))

    def verify(tag, r, v, t, method):
        ok = bool((t == STATUS_OK).all())
        if ok and method == METHOD_CALC_MULTIPLY:
            ok = bool(torch.equal(v, r.a0 * r.a1))
        if not ok:
            bad = int((t != STATUS_OK).sum())
            raise SystemExit(f"[rank {rank}] {tag}: verification failed ({bad} non-OK replies)")

    host_us_per_step = [None]
    host_split = [None]  # the sorted engine's host time split (timed steps, this rank)

    def measure(table, steps, warmup, delivery=args.delivery, sharding=args.sharding, Mq=M,
                method=METHOD_CALC_MULTIPLY, wide=False, pregen=False):
        """Warm up, then time `steps` Sends of `Mq` messages (barrier + synchronize
        on both sides, max over ranks); returns (seconds, exchange, graph used).
        Replies are verified after the warm-up and after the timed steps: every
        status OK and, for Calculator.Multiply, every value == A * B.  `pregen`:
        the batches are generated before the timing -- distinct ones, together
        more than the 256 MB MALL, cycled -- and each step is an eager Send."""
        pq = None
        if pregen:
            nb = max(3, -(-300_000_000 // (20 * Mq)))
            pq = [B.gen_requests(Mq, n_actors, METHOD_CALC_MULTIPLY, seed=(k * world + rank) * 104729 + 31,
                                 device=device) for k in range(nb)]
        # mailbox delivery: actor-sharded rings (each actor's messages in message
        # order in one ring) unless --sharding arrival (tile-sharded queues)
        ex = ActorExchange(table, Mq, chunks=chunks, state=state, fake=fake, delivery=delivery,
                           mailbox_ordered=sharding == "actor", mailbox_shards=args.mailbox_shards,
                           mailbox_slots=args.mailbox_slots, comm="ipc" if ipc else "rccl", group=G)
        _LIVE_EXCHANGES.append(weakref.ref(ex))  # (weak: a finished measurement's buffers stay freeable)
        if Mq == M and method == METHOD_CALC_MULTIPLY and not wide:
            rq, v, t = req, val, st
        else:
            # (SeqFold takes one argument: its batch carries no second column)
            rq = B.MsgBatch(torch.empty(Mq, dtype=torch.int32, device=device),
                            torch.empty(Mq, dtype=torch.int64, device=device),
                            None if method == METHOD_SEQ_FOLD else torch.empty(Mq, dtype=torch.int64, device=device),
                            None, method)
            v = torch.empty(Mq, dtype=torch.int64, device=device)
            t = torch.empty(Mq, dtype=torch.int32, device=device)
        graph = graph1 = None
        U = args.steps_per_graph
        vt = [rq, v, t]  # the batch and replies the verification reads
        if use_graph and pq is None:
            # the whole step (new requests + Send) as one hipGraph; the generator reads its
            # seed from device memory and the graph advances it, so every replay is a new batch
            seed_t = torch.tensor([rank * 0x9E3779B9 + 7 + j * 0x1000193 for j in range(U + 1)], dtype=torch.int64,
                                  device=device)

            def prologue(j=0):  # step j of a replay draws from seed j; the last one advances them all
                B.gen_requests(Mq, n_actors, method, wide=wide, device=device, out=rq, seed_tensor=seed_t[j:j + 1])
                if j == U - 1:
                    seed_t[:U].add_(U * 0x1000193)

            graph = ex.capture(rq, v, t, prologue=prologue, allow_collectives=args.graph == "on", repeat=U)
            if U > 1 and warmup % U:  # the warm-up steps a U-step replay cannot cover

                def prologue1(j=0):
                    B.gen_requests(Mq, n_actors, method, wide=wide, device=device, out=rq, seed_tensor=seed_t[U:U + 1])
                    seed_t[U:U + 1].add_(0x1000193)

                graph1 = ex.capture(rq, v, t, prologue=prologue1, allow_collectives=args.graph == "on", repeat=1)

        def step(s_):
            if graph is not None:
                if s_ < warmup and graph1 is not None:  # warm-up: one step per replay
                    graph1.replay()
                elif (s_ - warmup) % U == 0:  # timed: one replay runs U whole steps
                    graph.replay()
                return
            if pq is not None:
                ex.send_all(pq[s_ % len(pq)], out=(v, t))
                return
            if pre and Mq == M and method == METHOD_CALC_MULTIPLY:
                ex.send_all(pre[s_ % len(pre)], out=(v, t))
                return
            B.gen_requests(Mq, n_actors, method, wide=wide, seed=(s_ * world + rank) * 0x1000193 + 7, device=device, out=rq)
            ex.send(rq, v, t)

        def last(k):
            if pq is not None:
                return pq[(k - 1) % len(pq)]
            return pre[(k - 1) % len(pre)] if pre and Mq == M and method == METHOD_CALC_MULTIPLY else vt[0]

        for s_ in range(warmup):
            step(s_)
        sync()
        if warmup:
            verify("warmup", last(warmup), vt[1], vt[2], method)
        # re-send rounds are counted over the timed steps only: the first Sends of the
        # sorted exchange run at the static start-up capacity, before any agreement
        ex.warmup_resends, ex.counters.resends = ex.counters.resends, 0
        barrier()
        sync()
        sx = getattr(ex, "_sorted", None)
        prof0 = sx.host_profile() if sx is not None and hasattr(sx, "host_profile") else None
        t0 = time.perf_counter()
        host = 0.0
        for s_ in range(steps):
            h0 = time.perf_counter()
            step(warmup + s_)
            host += time.perf_counter() - h0
        sync()
        barrier()
        elapsed = time.perf_counter() - t0
        host_us_per_step[0] = host / max(steps, 1) * 1e6  # the host's time inside the step calls (no waits)
        if prof0 is not None:
            # where the host's step time goes: enqueueing the Send's work vs waiting for the
            # agreement of Send k - 2 (pick_spec: backpressure -- the host is 2 Sends ahead
            # of a busy GPU) vs resolving an overflow count
            p1 = sx.host_profile()
            d = {k: p1[k] - prof0[k] for k in p1}
            n = max(int(d.get("sends", 0)), 1)
            host_split[0] = {"sends": int(d.get("sends", 0)),
                             "enqueue_us_per_send": round((d["total_ns"] - d["spec_wait_ns"]) / n / 1e3, 2),
                             "agreement_wait_us_per_send": round(d["spec_wait_ns"] / n / 1e3, 2),
                             "overflow_wait_us_per_send": round(d["overflow_wait_ns"] / n / 1e3, 2)}
        elapsed = max_over_ranks(elapsed)
        if steps:
            verify("timed", last(warmup + steps), vt[1], vt[2], method)
        return elapsed, ex, graph is not None

    def mailbox_info(ex_):
        mb = ex_.mailboxes
        if mb is None:
            return {}
        # mailbox_shards: the rings allocated; ring_view_shards: how the timed Sends used them (stateless
        # batches: a coarser view of the same rings, every actor's messages still in one ring)
        # sharding_used: the rings the timed Sends took (a batch without ordered methods of up to
        # 2 Mi messages takes the arrival rings even when actor sharding is asked for)
        return {"sharding_used": getattr(mb, "last_sharding", None),
                "mailbox_shards": mb.shards, "ring_view_shards": mb.last_view_shards, "mailbox_slots": mb.slots,
                "mailbox_ring_bytes": mb.bytes, "mailbox_record_bytes": mb.last_record_bytes,
                "mailbox_route": mb.last_route}

    table = build_table(args.placement)
    hang_s = os.environ.get("PTYPE_HANG_DIAG")
    if hang_s is None and world > 1 and use_gpu:  # generous: RCCL set-up, secondaries, RTT calls included
        hang_s = str(300 + 0.2 * (args.steps + args.warmup) * (3 if not args.no_secondary else 1))
    if hang_s and float(hang_s) > 0:
        _hang_watchdog(float(hang_s), rank)
    head_method = METHOD_SEQ_FOLD if args.method == "seqfold" else METHOD_CALC_MULTIPLY
    elapsed, ex, graphed = measure(table, args.steps, args.warmup, method=head_method)
    head_host_us = host_us_per_step[0]
    head_host_split = host_split[0]
    def lookup_mode(t):
        if t.dir is None:
            return "hash-table probe"
        t.directory()
        return "computed (verified strided rule)" if t.affine else "route directory gather"

    route_mode = lookup_mode(table)
    head_mailbox = mailbox_info(ex)
    if head_mailbox.get("mailbox_route") == 3:  # the stateless mailbox Send resolved ranks only
        route_mode = "rank byte gather (1 B per id, from the route directory; stateless records carry the actor id)"
    elif head_mailbox.get("mailbox_route") == 4:
        route_mode = ("presence map in LDS (2 bits per id, folded from the route directory's rank bytes each Send; "
                      "stateless records carry the actor id)")
    secondaries = {}
    if args.placement != "affine" and not args.no_secondary and args.steps:
        # the same step with the strided placement, whose routes need no registry reads
        t2 = build_table("affine")
        e2, _, _ = measure(t2, args.steps, max(1, args.warmup))
        secondaries["affine_placement"] = {"placement": "affine", "registry_lookup": lookup_mode(t2),
                                           "delivery": args.delivery, "msgs_per_gpu_per_step": M,
                                           "value": M * world * args.steps / e2 if e2 > 0 else 0.0,
                                           "ms_per_step": e2 / args.steps * 1e3}
        del t2
    if world == 1 and not dist_on and fake is None and not args.no_secondary and args.steps:
        runs = []
        if args.delivery == "mailbox" and args.sharding == "actor":
            # BASELINE config 2 at its own size: 1 Mi messages per step
            runs.append(("config2_1m", dict(delivery="mailbox", sharding="actor", Mq=min(M, 1 << 20))))
            # the same 1 Mi step through arrival-sharded rings (stateless batches: a tile's messages in
            # one ring at fixed positions -- no sort, an enqueue and a drain kernel)
            runs.append(("config2_1m_arrival", dict(delivery="mailbox", sharding="arrival", Mq=min(M, 1 << 20))))
            # config 2 with the client's batches made before the timing (15 distinct 1 Mi batches,
            # 315 MB: more than the MALL), every step an eager Send through the actor-sharded rings
            runs.append(("config2_1m_pregen", dict(delivery="mailbox", sharding="actor", Mq=min(M, 1 << 20),
                                                   pregen=True)))
            # the headline step with the client's batches made before the timing (3 distinct 8 Mi
            # batches, 503 MB): the Send alone, eager
            runs.append(("mailbox_pregen", dict(delivery="mailbox", sharding="actor", pregen=True)))
            runs.append(("arrival_sharded", dict(delivery="mailbox", sharding="arrival")))
            # an ORDERED stateful method (SeqFold: state = state * K + a0, non-commutative):
            # every actor runs its messages one at a time in ring (= message) order
            runs.append(("ordered_seqfold", dict(delivery="mailbox", sharding="actor", method=METHOD_SEQ_FOLD)))
            # full-range int64 arguments: no 8-B ring record holds them (16-B records)
            runs.append(("wide_args", dict(delivery="mailbox", sharding="actor", wide=True)))
        if args.delivery != "direct":
            runs.append(("direct", dict(delivery="direct")))
        else:
            runs.append(("mailbox", dict(delivery="mailbox", sharding=args.sharding)))
        for name, kw in runs:
            e3, ex3, _ = measure(table, args.steps, max(1, args.warmup), **kw)
            Mq = kw.get("Mq", M)
            secondaries[name] = {"delivery": kw["delivery"], "placement": args.placement, "msgs_per_gpu_per_step": Mq,
                                 "value": Mq * args.steps / e3 if e3 > 0 else 0.0,
                                 "ms_per_step": e3 / args.steps * 1e3, **mailbox_info(ex3)}
            if kw["delivery"] == "mailbox":
                asked = kw.get("sharding", "actor")
                used = secondaries[name].get("sharding_used")
                secondaries[name]["sharding"] = asked if used in (None, asked) else (
                    f"{asked} asked; {used} rings used (a batch without ordered methods of <= 2 Mi messages)")
                secondaries[name]["method"] = "SeqFold (ordered)" if kw.get("method") == METHOD_SEQ_FOLD \
                    else "Calculator.Multiply"
                secondaries[name]["args"] = "full-range int64" if kw.get("wide") else "A: 16-bit signed, B: 16-bit"
                if kw.get("pregen"):
                    nb = max(3, -(-300_000_000 // (20 * Mq)))
                    secondaries[name]["batches"] = (f"{nb} distinct pre-generated batches ({nb * 20 * Mq >> 20} MB), "
                                                    "cycled; eager Sends, generator not in the timed steps")
            del ex3

    # BASELINE configs 4 and 5 and the public API path, under the same clock (utils/benchmarks.py)
    if not args.no_secondary and args.steps and use_gpu and fake is None:
        from ptype_amd.utils import benchmarks as BM

        secondaries["optimus_fanout"] = BM.optimus_fanout(table, n_actors, device, args.steps, max(1, args.warmup),
                                                          rank=rank, world=world, chunks=chunks,
                                                          comm="ipc" if ipc else "rccl",
                                                          barrier=barrier if dist_on else None,
                                                          max_over_ranks=max_over_ranks, group=G)
        if world == 1 and not dist_on:  # one process: a failing secondary is reported, the headline kept
            for name, fn in (("registry_1m", lambda: BM.registry_1m(device)),
                             ("api_send", lambda: BM.api_send(device, sorted({M, min(M, 1 << 20)}, reverse=True),
                                                              args.actors_per_gpu, args.steps, max(1, args.warmup)))):
                try:
                    secondaries[name] = fn()
                except Exception as e:  # noqa: BLE001
                    secondaries[name] = {"error": f"{type(e).__name__}: {e}"[:300]}
                    print(f"[bench] secondary {name} failed: {e!r}", file=sys.stderr, flush=True)

    # p50 RTT of a synchronous Call to a GPU actor (persistent dispatcher, no kernel
    # launch per call): from this process to its own GPU, and -- with more than one
    # rank -- from this process to the actors of the NEXT rank's GPU, through that
    # process's shared-memory rings (the reference's Client.Call to another node,
    # cluster/rpc.go:59-67; here a node is a GPU of the same host)
    p50 = p50_remote = None
    ring_on_device = None
    remote_ring = None
    rtt_errors: list[str] = []
    if use_gpu and args.rtt_calls > 0 and fake is None:
        from ptype_amd.ops import hip

        tag = os.environ.get("MASTER_PORT", "0")
        shm = f"/ptype-bench-{tag}-{rank}" if dist_on else ""
        srv = hip().DeviceServer(device.index, 4096, state.data_ptr(), state.numel(), 0, 200.0, 60.0, shm)

        def timed_calls(call):
            lat = []
            for i in range(args.rtt_calls + 100):
                a = i % state.numel()
                t = time.perf_counter()
                v, s_ = call(METHOD_CALC_MULTIPLY, a, i, 3)[:2]
                dt = time.perf_counter() - t
                if v != 3 * i or s_ != STATUS_OK:
                    raise RuntimeError(f"RTT call returned {v}, status {s_}")
                if i >= 100:
                    lat.append(dt)
            lat.sort()
            return lat[len(lat) // 2] * 1e6

        ring_on_device = bool(srv.ring_on_device)
        # a failed call is reported, never raised between the barriers: the other
        # ranks would wait there forever
        try:
            p50 = timed_calls(srv.call)
        except Exception as e:
            rtt_errors.append(f"local: {e}")
            p50 = -1.0
        if dist_on:
            from ptype_amd import _core

            # host-side barriers through the rendezvous store: no collective kernel
            # sits on any GPU while the peers' dispatchers must (re)launch to serve
            def host_barrier(key):
                BM.kv_barrier(bench_cp, key, world)

            host_barrier("ptype/bench/rtt/ready")  # every rank's dispatcher segment exists
            try:
                peer = _core.ShmClient(f"/ptype-bench-{tag}-{(rank + 1) % world}")
                remote_ring = peer.ring_placement
                p50_remote = timed_calls(peer.call)
            except Exception as e:
                rtt_errors.append(f"remote: {e}")
                p50_remote = -1.0
            host_barrier("ptype/bench/rtt/done")  # keep serving until every rank is done calling
        srv.close()
        if dist_on:
            n_err = max_over_ranks(float(len(rtt_errors)))
            p50, p50_remote = max_over_ranks(max(p50, 0.0)), max_over_ranks(max(p50_remote or 0.0, 0.0))
            if n_err and not rtt_errors:
                rtt_errors.append("on another rank")
        if rtt_errors:
            p50 = p50_remote = None

    total_msgs = M * world * args.steps
    value = total_msgs / elapsed if elapsed > 0 else 0.0
    printed = [False]

    def emit():  # rank 0's one JSON line (also from the hang watchdog, once, after a late secondary hangs)
        if rank != 0 or printed[0]:
            return
        printed[0] = True
        out = {
            "metric": "messages/sec",
            "value": value,
            "unit": "msg/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / max(args.steps, 1) * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            # the cross-GPU call when there is another GPU, else the local one
            "p50_rtt_us": p50_remote if world > 1 else p50,
            "p50_rtt_local_us": p50,
            "p50_rtt_remote_us": p50_remote,
            "rtt_path": "host -> GPU actor via the persistent dispatcher's rings (remote: the next rank's "
                        "process: its GPU's request ring mapped from a dma-buf, replies in shared memory)",
            "rtt_request_ring": None if ring_on_device is None else ("device (host writes via BAR)" if ring_on_device
                                                                      else "pinned host"),
            # remote: the next rank's GPU ring, mapped here from its dma-buf ("device") or its shm segment
            "rtt_remote_request_ring": remote_ring,
            "rtt_error": "; ".join(rtt_errors) if rtt_errors else None,
            "config": {
                "model": "calculator actor (Calculator.Multiply)" if args.method == "multiply" else
                         "SeqFold actor (ordered stateful method; experiment, not the headline)",
                "global_batch": M * world,
                "seq_len": None,
                "parallelism": (f"{world} ranks sharing {torch.cuda.device_count()} GPU(s), IpcComm all-to-alls "
                                "(multi-process rehearsal, not a scaling figure)" if ipc else
                                f"actors sharded over {world} GPU(s)" + ((", RCCL all-to-all epochs" if use_gpu
                                                                          else ", gloo all-to-all epochs (CPU)")
                                                                         if dist_on else "")),
                # the N > 1 communicator: the compiled DataPlane's (Join's), never a torch process group's
                "comm": (("DataPlane/IpcComm" if ipc else "DataPlane/RCCL") if native else
                         ("gloo" if dist_on else None)),
                "msgs_per_gpu_per_step": M,
                "actors": n_actors,
                "chunks": chunks,
                **wire_info(ex, req),
                "client_batch": "SoA (actor u32, A i64, B i64)",
                "args": "A: 16-bit signed, B: 16-bit (int64 columns; see secondaries.wide_args for full-range)",
                "hip_graph": graphed,
                "steps_per_graph": args.steps_per_graph if graphed else None,
                # host time inside the timed step calls (this rank; a graph replay launches U steps)
                "host_us_per_step": round(head_host_us, 2) if head_host_us is not None else None,
                **({"host_split": head_host_split} if head_host_split is not None else {}),
                **({"load": f"zipf({args.zipf})" if args.zipf > 0 else "uniform", "pregenerated": True,
                    "resend_rounds": ex.counters.resends, "resend_rounds_warmup": ex.warmup_resends}
                   if pregen else {}),
                **({"slot_capacity": ex.last_wire.get("C"), "slot_capacity_alloc": ex.last_wire.get("C_alloc"),
                    "slot_capacity_static": ex.C} if ex.last_wire is not None else {}),
                "placement": args.placement,
                "registry_lookup": route_mode,
                "delivery": args.delivery,
                **({"sharding": args.sharding, **head_mailbox} if args.delivery == "mailbox" else {}),
                **({"loopback_ranks": args.loopback, "link_gbps": args.link_gbps, "note": "profiling mode: rank 0 of a symmetric "
                    f"{args.loopback}-rank node, all-to-alls as local copies (not a headline number)"}
                   if fake else {}),
            },
        }
        if secondaries:
            out["secondaries"] = secondaries
        print(json.dumps(out), flush=True)

    if dist_on and use_gpu and fake is None and not args.no_secondary and args.steps:
        # the public API path at N > 1 (Join -> NewClient -> Client.Send on every rank), last: if it
        # hangs, the hang watchdog prints the line measured so far (emit) instead of nothing
        from ptype_amd.utils import benchmarks as BM

        secondaries["api_send"] = {"error": "did not finish (hang watchdog)"}
        _EMIT_ON_HANG[0] = emit
        try:
            secondaries["api_send"] = BM.api_send(device, [min(M, 1 << 22)], args.actors_per_gpu, args.steps,
                                                  max(1, args.warmup), rank=rank, world=world,
                                                  comm="ipc" if ipc else "rccl", barrier=barrier,
                                                  max_over_ranks=max_over_ranks)
        except Exception as e:  # noqa: BLE001
            secondaries["api_send"] = {"error": f"{type(e).__name__}: {e}"[:300]}
            print(f"[rank {rank}] secondary api_send failed: {e!r}", file=sys.stderr, flush=True)
    emit()
    if native:
        G.close()
        bench_cp.Close()
    elif dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""route_prep variants on the directory path (random placement): items per
thread x software-pipelined actor loads, one chunk of M messages, R ranks.
Times the whole 3-pass route (prep + scan + packed scatter) with hipEvents;
run under rocprofv3 --kernel-trace --stats for the prep kernel alone.
usage: python tools/prep_sweep.py [M] [R,R,...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ptype_amd import ops  # noqa: E402
from ptype_amd.ops import batch as B  # noqa: E402
from ptype_amd.ops import packed as P  # noqa: E402
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY  # noqa: E402
from ptype_amd.ops.table import RegistryTable, actor_keys  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


M = int(sys.argv[1]) if len(sys.argv) > 1 else 4 << 20
RS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 8]
for R in RS:
    n = 131072 * R
    g = RegistryTable(2 * n, device="cuda")
    ids = torch.arange(n)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(5))
    g.upsert(actor_keys(ids), (perm % R).to(torch.int32), (perm // R).to(torch.int32))
    g.enable_directory(n)  # random placement: every message gathers its route word
    req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=1, device="cuda")
    L = P.layout(P.meta_list(P.meta(req, g)))
    C = B.stripe_capacity(M, R, 0.01)
    rws = B.RouteWorkspace(M, R, "cuda")
    send = torch.empty(R * P.req_words(C, L["S"]), dtype=torch.int32, device="cuda")
    ref = None
    for items, pipe in ((2, -1), (4, -1), (8, -1), (2, 0), (4, 0), (8, 0)):
        ops.hip().set_route_tuning(items, 0, pipe)
        try:
            t = timed(lambda: P.route(req, g, R, C, L, rank_self=0, sendbuf=send, rws=rws))
            P.route(req, g, R, C, L, rank_self=0, sendbuf=send, rws=rws)
            torch.cuda.synchronize()
            out = send.clone()
        finally:
            ops.hip().set_route_tuning(0, 0, 0)
        ok = True if ref is None else bool(torch.equal(out, ref))
        ref = out if ref is None else ref
        print(json.dumps({"R": R, "M": M, "items": items, "pipe": pipe, "route_us": round(t, 1), "same": ok}),
              flush=True)

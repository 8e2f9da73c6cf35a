#!/usr/bin/env python3
"""Per-stage timing of the Send pipeline on one GPU (hipEvent brackets).

Sweeps registry size x route_prep variant (items per thread, hash probe vs
route directory) and reports route (prep+scan+scatter), dispatch and complete
in microseconds for an 8 Mi-message batch.  Used to pick the defaults in
csrc/hip/batch.hip; results are logged in profiles/README.md.

usage: python tools/route_bench.py [--msgs N] [--iters K]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ptype_amd.ops import batch as B, hip  # noqa: E402
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY  # noqa: E402
from ptype_amd.ops.table import RegistryTable, actor_keys  # noqa: E402


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--msgs", type=int, default=8 << 20)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--ranks", type=int, default=1)
    p.add_argument("--full", action="store_true", help="32-B records (FULL_FORMAT) instead of the batch's format")
    p.add_argument("--sizes", default="4096,131072,1048576")
    a = p.parse_args()
    M, R = a.msgs, a.ranks
    C = B.stripe_capacity(M, R)
    rows = []
    for n_actors in [int(x) for x in a.sizes.split(",")]:
        t = RegistryTable(2 * n_actors, device="cuda")
        ids = torch.arange(n_actors, dtype=torch.int64)
        t.upsert(actor_keys(ids), (ids % R).to(torch.int32), (ids // R).to(torch.int32))
        req = B.gen_requests(M, n_actors, METHOD_CALC_MULTIPLY, seed=5, device="cuda")
        fmt = B.WireFormat.for_batch(req) if not a.full else B.FULL_FORMAT
        send = torch.empty(R * fmt.req_words(C), dtype=torch.int32, device="cuda")
        perm = torch.empty(M, dtype=torch.int32, device="cuda")
        rws = B.RouteWorkspace(M, R, "cuda")
        reply = torch.empty(R * B.WireFormat.rep_words(C), dtype=torch.int32, device="cuda")
        val = torch.empty(M, dtype=torch.int64, device="cuda")
        st = torch.empty(M, dtype=torch.int32, device="cuda")
        for use_dir in (False, True, "affine"):
            if use_dir:
                t.enable_directory(n_actors, affine_world=R if use_dir == "affine" else 0)
            for mode, items in ((1, 0), (0, 1), (0, 2), (0, 4)):
                hip().set_route_tuning(items, mode)
                us = timed(lambda: B.route(req, t, R, C, sendbuf=send, perm=perm, rws=rws, fmt=fmt), a.iters)
                rows.append({"actors": n_actors, "dir": use_dir, "route": "single-pass" if mode == 1 else "3-pass",
                             "items": items, "route_us": round(us, 1)})
            hip().set_route_tuning(0, 0)
            t.dir = None
        d_us = timed(lambda: B.dispatch(send, R, C, reply=reply, ws=rws.ws, expected_per_rank=M // R,
                                          fmt=fmt), a.iters)
        c_us = timed(lambda: B.complete(reply, perm, C, val, st), a.iters)
        g_us = timed(lambda: B.gen_requests(M, n_actors, METHOD_CALC_MULTIPLY, seed=6, device="cuda", out=req),
                     a.iters)
        rows.append({"actors": n_actors, "ranks": R, "fmt_stride_words": fmt.stride, "gen_us": round(g_us, 1), "dispatch_us": round(d_us, 1),
                     "complete_us": round(c_us, 1)})
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()

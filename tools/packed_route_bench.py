"""Wire-v3 route (prep + scan + packed scatter), dispatch and complete vs rank count,
one chunk of M messages on one GPU (the destinations are slot regions in HBM; no
collective).  usage: python tools/packed_route_bench.py [M] [R,R,...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

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


M = int(sys.argv[1]) if len(sys.argv) > 1 else 2 * 1024 * 1024
RS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 8]
for R in RS:
    n = 131072 * R
    g = RegistryTable(2 * n, device="cuda")
    ids = torch.arange(n)
    g.upsert(actor_keys(ids), (ids % R).to(torch.int32), (ids // R).to(torch.int32))
    g.enable_directory(n, affine_world=R)
    req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=1, device="cuda")
    L = P.layout(P.meta_list(P.meta(req, g)))
    C = B.stripe_capacity(M, R, 0.01)
    rws = B.RouteWorkspace(M, R, "cuda")
    send = torch.empty(R * P.req_words(C, L["S"]), dtype=torch.int32, device="cuda")
    t_route = timed(lambda: P.route(req, g, R, C, L, rank_self=0, sendbuf=send, rws=rws))
    _, perm, _ = P.route(req, g, R, C, L, rank_self=0, sendbuf=send, rws=rws)
    rep = P.dispatch(send, R, C, L)
    t_disp = timed(lambda: P.dispatch(send, R, C, L))
    t_comp = timed(lambda: P.complete(rep, perm, C, L["vb"]))
    val, st = P.complete(rep, perm, C, L["vb"])
    ok = bool(torch.equal(val, req.a0 * req.a1)) and bool((st == 0).all())
    print(json.dumps({"R": R, "M": M, "route_us": round(t_route, 1), "dispatch_us": round(t_disp, 1),
                      "complete_us": round(t_comp, 1), "S": L["S"], "vb": L["vb"], "ok": ok}), flush=True)

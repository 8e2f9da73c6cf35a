#!/usr/bin/env python3
"""Python-side host cost of one N > 1 Send (loopback-8 sorted exchange, 1 Mi
messages): wall time of ActorExchange.send vs the native SortedExchange.send
inside it (host_profile), plus a cProfile of the Python frames.  One JSON line
and the profile's top entries on stderr."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ptype_amd.ops import batch as B  # noqa: E402
from ptype_amd.ops import hip  # noqa: E402
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY  # noqa: E402
from ptype_amd.ops.table import RegistryTable, actor_keys  # noqa: E402
from ptype_amd.parallel.exchange import ActorExchange  # noqa: E402


def main():
    R, M, n = 8, 1 << 20, 131072 * 8
    dev = torch.device("cuda", 0)
    tab = RegistryTable(2 * n, device=dev)
    ids = torch.arange(n)
    slot = torch.randperm(n, generator=torch.Generator().manual_seed(5))
    tab.upsert(actor_keys(ids), (slot % R).to(torch.int32), (slot // R).to(torch.int32))
    tab.enable_directory(n)
    ex = ActorExchange(tab, M, chunks=2, state=torch.zeros(n // R, dtype=torch.int64, device=dev),
                       fake=(hip().FakeComm(R, loopback=True), 0), delivery="mailbox", mailbox_ordered=False)
    req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=1, device=dev)
    val = torch.empty(M, dtype=torch.int64, device=dev)
    st = torch.empty(M, dtype=torch.int32, device=dev)
    for _ in range(10):
        ex.send(req, val, st)
    torch.cuda.synchronize()
    p0 = ex._sorted.host_profile()
    N = 200
    t = time.perf_counter()
    for _ in range(N):
        ex.send(req, val, st)
    wall = (time.perf_counter() - t) / N
    torch.cuda.synchronize()
    p1 = ex._sorted.host_profile()
    native = (p1["total_ns"] - p0["total_ns"]) / N / 1e3
    wait = (p1["spec_wait_ns"] - p0["spec_wait_ns"]) / N / 1e3
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(N):
        ex.send(req, val, st)
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
    print(s.getvalue(), file=sys.stderr)
    print(json.dumps({"send_wall_us": round(wall * 1e6, 2), "native_us": round(native, 2),
                      "native_agreement_wait_us": round(wait, 2),
                      "python_us": round(wall * 1e6 - native, 2)}), flush=True)


if __name__ == "__main__":
    main()

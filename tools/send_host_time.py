#!/usr/bin/env python3
"""Host time per Client.Send: the DeviceRuntime data-plane Send
of a 1 Mi-message batch at world 1 (mailbox delivery), timed on the host with
no synchronisation inside the loop -- what the caller's thread spends to
enqueue one Send -- next to the GPU time per Send.  Also a cProfile of the
Python frames on the path.  Prints one JSON line."""
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
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY  # noqa: E402
from ptype_amd.runtime import DeviceRuntime  # noqa: E402


def main():
    M = int(os.environ.get("SEND_M", 1 << 20))
    delivery = os.environ.get("SEND_DELIVERY", "mailbox")
    rt = DeviceRuntime(torch.device("cuda", 0), actors=1 << 17, service="calc", max_batch=M, delivery=delivery)
    rt.place_local()
    req = B.gen_requests(M, rt.total_actors, METHOD_CALC_MULTIPLY, seed=1, device="cuda")
    for _ in range(5):
        rt.send("calc", req)
    torch.cuda.synchronize()
    steps = 200
    host = 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        h = time.perf_counter()
        rt.send("calc", req)
        host += time.perf_counter() - h
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    layers = {}
    if delivery == "mailbox":  # host time of each layer of the path, innermost first
        ex = rt.exchange
        mb = ex.mailboxes
        from ptype_amd.ops import _ptr

        d, n_dir, affine = rt.table.directory()
        val = torch.empty(M, dtype=torch.int64, device="cuda")
        st = torch.empty(M, dtype=torch.int32, device="cuda")
        args = (_ptr(req.actor), _ptr(req.a0), _ptr(req.a1), 0, 0, int(req.method), M, _ptr(rt.table.table),
                rt.table.cap, _ptr(d), n_dir, affine, 0, 0, _ptr(val), _ptr(st), M, _ptr(rt.state), rt.state.numel(),
                0, [], 0, False, False, int(req.method), mb._stream())

        def timeit(fn, k=200):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(k):
                fn()
            h = (time.perf_counter() - t) / k
            torch.cuda.synchronize()
            return round(h * 1e6, 2)

        layers["native_send_sorted"] = timeit(lambda: mb._m.send_sorted(*args))
        layers["Mailboxes.send"] = timeit(lambda: mb.send(req, rt.table, rt.state, val, st, ordered=False))
        layers["ActorExchange.send"] = timeit(lambda: ex.send(req, val, st))
        layers["ActorExchange.send_all"] = timeit(lambda: ex.send_all(req))
        layers["DeviceRuntime.send"] = timeit(lambda: rt.send("calc", req))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(50):
        rt.send("calc", req)
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(12)
    out = {"M": M, "host_us_per_send": round(host / steps * 1e6, 2), "wall_us_per_send": round(wall / steps * 1e6, 2),
           "delivery": delivery, "path": "DeviceRuntime.send -> send_all -> " + delivery,
           "host_us_by_layer": layers,
           "mailbox_stats": rt.exchange.mailboxes.stats() if rt.exchange.mailboxes is not None else None}
    print(s.getvalue()[-3000:], file=sys.stderr)
    print(json.dumps(out))
    rt.close()


if __name__ == "__main__":
    main()

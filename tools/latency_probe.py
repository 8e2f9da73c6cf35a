#!/usr/bin/env python3
"""Single-call latency breakdown of the persistent dispatcher on one GPU:
host round trip (log2 histogram), device queue (publish -> picked up) and
service (picked up -> reply) time from the s_memrealtime trace ring."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ptype_amd.ops import hip  # noqa: E402
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY  # noqa: E402
from ptype_amd.utils import trace  # noqa: E402


def main(n=5000):
    state = torch.zeros(1024, dtype=torch.int64, device="cuda")
    srv = hip().DeviceServer(0, 4096, state.data_ptr(), 1024, 0, 500.0, 60.0)
    try:
        for i in range(200):
            srv.call(METHOD_CALC_MULTIPLY, i, i, 3)
        lat = []
        with trace.DispatcherTrace(srv, capacity=8192) as t:
            for i in range(n):
                t0 = time.perf_counter()
                srv.call(METHOD_CALC_MULTIPLY, i % 1024, i, 3)
                lat.append((time.perf_counter() - t0) * 1e6)
            b = t.breakdown()
        b["python_call_us"] = trace.percentiles(lat)
        lat = []  # the same loop with tracing off (what bench.py measures)
        for i in range(n):
            t0 = time.perf_counter()
            srv.call(METHOD_CALC_MULTIPLY, i % 1024, i, 3)
            lat.append((time.perf_counter() - t0) * 1e6)
        b["python_call_untraced_us"] = trace.percentiles(lat)
        print(json.dumps(b))
    finally:
        srv.close()


if __name__ == "__main__":
    main()

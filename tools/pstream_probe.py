#!/usr/bin/env python3
"""Diagnose persistent kernels vs other streams (run on the GPU box).

A DeviceServer wave is made resident (idle exit after IDLE s); then, on each of
N fresh torch streams, one in-place add runs and that stream is synchronised.
Prints per-stream wall time and the value each stream reads back, the server's
running flag, and the totals after a device-wide synchronise.  Compare
PTYPE_TUNE=persistent_stream=low (default) / high / cumask / pooled (common.hpp
dedicated_stream)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ptype_amd.ops import hip  # noqa: E402
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY  # noqa: E402

IDLE_MS = float(os.environ.get("IDLE_MS", "3000"))
N = int(os.environ.get("NSTREAMS", "40"))


def main():
    dev = torch.device("cuda", 0)
    state = torch.zeros(64, dtype=torch.int64, device=dev)
    x = torch.zeros(1024, device=dev)
    torch.cuda.synchronize()
    srv = hip().DeviceServer(0, 256, state.data_ptr(), state.numel(), 0, IDLE_MS, 30.0, "")
    print(json.dumps({"mode": os.environ.get("PTYPE_TUNE", "persistent_stream=low"),
                      "first_call": list(srv.call(METHOD_CALC_MULTIPLY, 1, 6, 7)), "running": srv.running,
                      "wave_stream_priority": srv.stream_priority}), flush=True)
    rows = []
    for k in range(N):
        s = torch.cuda.Stream(dev)
        t = time.perf_counter()
        with torch.cuda.stream(s):
            x.add_(1)
            v = float(x[0].item())  # copy on s: waits for s's add
        dt = time.perf_counter() - t
        rows.append({"k": k, "stream": hex(s.cuda_stream), "ms": round(dt * 1e3, 2), "x": v, "running": srv.running})
        print(json.dumps(rows[-1]), flush=True)
    # legacy default (null) stream work while the wave is resident
    t = time.perf_counter()
    y = torch.ones(1024, device=dev) * 3
    yv = float(y[0].item())
    print(json.dumps({"null_stream_ms": round((time.perf_counter() - t) * 1e3, 2), "y": yv, "running": srv.running}),
          flush=True)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (None, None)
    print(json.dumps({"torch_priority_range": [lo, hi]}), flush=True)
    t = time.perf_counter()
    torch.cuda.synchronize()
    print(json.dumps({"device_sync_ms": round((time.perf_counter() - t) * 1e3, 2), "x_final": float(x[0]),
                      "running": srv.running}), flush=True)
    srv.close()


if __name__ == "__main__":
    main()

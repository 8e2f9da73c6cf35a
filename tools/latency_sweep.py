"""Single-call latency vs the dispatcher's polling knobs (tune poll_lanes / poll_full /
_SLEEP, read when a DeviceServer is built), all in one process on one box so the
variants are comparable.  Prints one JSON line per variant."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ptype_amd.ops import hip  # noqa: E402
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY  # noqa: E402

VARIANTS = [(64, 1, 1), (64, 0, 1), (16, 1, 1), (16, 0, 1), (1, 1, 1), (64, 1, 8), (64, 0, 8), (1, 1, 8),
            (64, 1, 1)]
state = torch.zeros(1024, dtype=torch.int64, device="cuda")
for lanes, full, sleep in VARIANTS:
    os.environ["PTYPE_TUNE"] = f"poll_lanes={lanes},poll_full={full},poll_sleep={sleep}"
    srv = hip().DeviceServer(0, 4096, state.data_ptr(), 1024, 0, 500.0, 60.0)
    try:
        for i in range(300):
            srv.call(METHOD_CALC_MULTIPLY, i % 1024, i, 3)
        lat = []
        for i in range(4000):
            t0 = time.perf_counter()
            v, s, _ = srv.call(METHOD_CALC_MULTIPLY, i % 1024, i, 3)
            lat.append((time.perf_counter() - t0) * 1e6)
            assert v == 3 * i and s == 0
        lat.sort()
        print(json.dumps({"lanes": lanes, "full": full, "sleep": sleep, "p50_us": round(lat[len(lat) // 2], 3),
                          "p90_us": round(lat[int(len(lat) * 0.9)], 3), "p99_us": round(lat[int(len(lat) * 0.99)], 3)}),
              flush=True)
    finally:
        srv.close()

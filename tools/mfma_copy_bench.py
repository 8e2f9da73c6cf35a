#!/usr/bin/env python3
"""AoS -> SoA of 32-B records: dwordx4 copy vs MFMA byte transposition (SURVEY
7.4.8 / the north star's "MFMA-packed batch copies").  Times both on 16 Mi
records with hipEvents; run under rocprofv3 for counters."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ptype_amd.ops import batch as B  # noqa: E402
from ptype_amd.ops.records import make_requests  # noqa: E402


def main(M=16 << 20, iters=20):
    g = torch.Generator(device="cuda").manual_seed(1)
    cols = [torch.randint(0, 1 << 30, (M,), device="cuda", generator=g) for _ in range(5)]
    req = make_requests(*cols)
    out = {}
    for mfma in (False, True):
        B.MsgBatch.from_records(req, mfma=mfma)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            B.MsgBatch.from_records(req, mfma=mfma)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / iters
        moved = M * (32 + 4 + 2 + 24)
        out["mfma" if mfma else "dwordx4_copy"] = {"us": round(us, 1), "GB_per_s": round(moved / us / 1e3, 1)}
    print(json.dumps({"records": M, **out}))


if __name__ == "__main__":
    main()

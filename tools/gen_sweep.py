#!/usr/bin/env python3
"""Synthetic-client generator: time per batch (hipEvents) and bit-exactness vs the
CPU reference.  Variants are selected by env (PTYPE_GEN_DIV, PTYPE_GEN_BLOCKS),
so run one process per variant.  usage: python tools/gen_sweep.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ptype_amd.ops import batch as B  # noqa: E402

for M in (1 << 20, 8 << 20):
    n = 131072
    out = B.gen_requests(M, n, seed=3, device="cuda")
    ref = B.gen_requests(1 << 16, 1_000_003, seed=7, device="cpu")
    chk = B.gen_requests(1 << 16, 1_000_003, seed=7, device="cuda")
    same = all(torch.equal(getattr(chk, c).cpu(), getattr(ref, c)) for c in ("actor", "a0", "a1"))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        B.gen_requests(M, n, seed=3, device="cuda", out=out)
    e0.record()
    for k in range(50):
        B.gen_requests(M, n, seed=k, device="cuda", out=out)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"M": M, "div": os.environ.get("PTYPE_GEN_DIV", "0"), "blocks": os.environ.get("PTYPE_GEN_BLOCKS", "8192"),
                      "us": round(e0.elapsed_time(e1) / 50 * 1e3, 2), "exact": same}), flush=True)

#!/usr/bin/env python3
"""The request generator alone, back to back (no other kernel between): its kernel
time at 1 Mi and 8 Mi, under rocprofv3 --kernel-trace --stats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ptype_amd.ops import batch as B  # noqa: E402
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY  # noqa: E402

for M in (1 << 20, 8 << 20):
    rq = B.MsgBatch(torch.empty(M, dtype=torch.int32, device="cuda"), torch.empty(M, dtype=torch.int64, device="cuda"),
                    torch.empty(M, dtype=torch.int64, device="cuda"), None, METHOD_CALC_MULTIPLY)
    for k in range(20):
        B.gen_requests(M, 131072, METHOD_CALC_MULTIPLY, seed=k, device="cuda", out=rq)
    torch.cuda.synchronize()
print("ok")

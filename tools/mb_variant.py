#!/usr/bin/env python3
"""One mailbox Send variant at the bench's size, for per-kernel profiles:
actor (per-actor rings, Calculator.Multiply), arrival (tile rings), seqfold
(ordered SeqFold on per-actor rings).  usage: mb_variant.py VARIANT [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ptype_amd.ops import batch as B  # noqa: E402
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_SEQ_FOLD  # noqa: E402
from ptype_amd.ops.table import RegistryTable, actor_keys  # noqa: E402
from ptype_amd.parallel.exchange import ActorExchange  # noqa: E402


def main():
    variant = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    M, n = int(os.environ.get("MB_M", 8 << 20)), 131072
    S = int(os.environ.get("MB_SHARDS", 256))
    dev = torch.device("cuda", 0)
    t = RegistryTable(2 * n, device=dev)
    affine = os.environ.get("MB_AFFINE") == "1"  # identity placement: routes computed, no directory gather
    perm = torch.arange(n) if affine else torch.randperm(n, generator=torch.Generator().manual_seed(1))
    t.upsert(actor_keys(torch.arange(n)), torch.zeros(n, dtype=torch.int32), perm.to(torch.int32))
    t.enable_directory(n, affine_world=1)
    state = torch.zeros(n, dtype=torch.int64, device=dev)
    ex = ActorExchange(t, M, chunks=1, state=state, delivery="mailbox", mailbox_shards=S,
                       mailbox_ordered=variant != "arrival")
    method = METHOD_SEQ_FOLD if variant == "seqfold" else METHOD_CALC_MULTIPLY
    req = B.gen_requests(M, n, method, seed=3, device=dev)
    val = torch.empty(M, dtype=torch.int64, device=dev)
    st = torch.empty(M, dtype=torch.int32, device=dev)
    for _ in range(3):
        ex.send(req, val, st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ex.send(req, val, st)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"{variant}: {dt * 1e3:.4f} ms/send, {M / dt / 1e9:.1f} G msg/s")


if __name__ == "__main__":
    main()

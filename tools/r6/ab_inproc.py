#!/usr/bin/env python3
"""In-process A/B of the 8 Mi stateless mailbox step: actor-sharded sort vs arrival
rings, alternated in ONE process (same table, same warm GPU), each timed as the
bench times its headline (20 steps per hipGraph replay, generator in the step)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import bench  # noqa: E402
from ptype_amd.ops import batch as B  # noqa: E402
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, STATUS_OK  # noqa: E402
from ptype_amd.ops.table import RegistryTable, actor_keys  # noqa: E402
from ptype_amd.parallel import exchange as X  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    M, n = 8 << 20, 131072
    t = RegistryTable(2 * n, device=dev)
    r, mb = bench.place_actors(n, 1, "random")
    t.upsert(actor_keys(torch.arange(n)), r, mb)
    t.enable_directory(n, affine_world=1)
    state = torch.zeros(n, dtype=torch.int64, device=dev)
    out = []
    for rep in range(3):
        for mode in ("actor", "arrival"):
            X.ARRIVAL_AUTO_MAX = (64 << 20) if mode == "arrival" else (2 << 20)
            ex = X.ActorExchange(t, M, state=state, delivery="mailbox", mailbox_ordered=True)
            req = B.MsgBatch(torch.empty(M, dtype=torch.int32, device=dev), torch.empty(M, dtype=torch.int64, device=dev),
                             torch.empty(M, dtype=torch.int64, device=dev), None, METHOD_CALC_MULTIPLY)
            v = torch.empty(M, dtype=torch.int64, device=dev)
            st = torch.empty(M, dtype=torch.int32, device=dev)
            seed = torch.tensor([rep * 977 + j * 0x1000193 for j in range(21)], dtype=torch.int64, device=dev)

            def prologue(j=0):
                B.gen_requests(M, n, METHOD_CALC_MULTIPLY, device=dev, out=req, seed_tensor=seed[j:j + 1])
                if j == 19:
                    seed[:20].add_(20 * 0x1000193)

            g = ex.capture(req, v, st, prologue=prologue, repeat=20)
            g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 20 * 1e3
            ok = bool((st == STATUS_OK).all()) and torch.equal(v, req.a0 * req.a1)
            used = ex.mailboxes.last_sharding
            out.append({"rep": rep, "mode": mode, "used": used, "ms_per_step": round(ms, 4),
                        "G_msg_s": round(M / ms / 1e6, 2), "ok": ok})
            print(json.dumps(out[-1]), flush=True)
            del g, ex


if __name__ == "__main__":
    main()

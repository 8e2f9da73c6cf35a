#!/usr/bin/env python3
"""Host enqueue cost of ActorExchange.send vs its GPU time (single rank, RCCL
forced on so the collective calls are real), for the native epoch engine and
the Python pipeline (tune engine=0 path).  If the enqueue time per step
approaches the GPU time, the multi-GPU step is host-bound.  Also checks that
both paths return identical results."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ptype_amd.ops import batch as B  # noqa: E402
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY  # noqa: E402
from ptype_amd.ops.table import RegistryTable, actor_keys  # noqa: E402
from ptype_amd.parallel.exchange import ActorExchange  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    n, M = 131072, 8 << 20
    t = RegistryTable(2 * n, device=dev)
    ids = torch.arange(n)
    t.upsert(actor_keys(ids), torch.zeros(n, dtype=torch.int32), ids.to(torch.int32))
    t.enable_directory(n, affine_world=1)
    out = {}
    req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=1, device=dev)
    variants = (("engine_rccl", True, True), ("engine_local", True, False), ("python_rccl", False, True))
    for chunks in (1, 2, 4, 8):
        res = {}
        for name, engine, coll in variants:
            ex = ActorExchange(t, M, chunks=chunks)
            ex.use_engine, ex.force_collectives = engine, coll
            val = torch.empty(M, dtype=torch.int64, device=dev)
            st = torch.empty(M, dtype=torch.int32, device=dev)
            for _ in range(3):
                ex.send(req, val, st)
            torch.cuda.synchronize()
            if ex._engine is not None:
                ex._engine.reset_host_profile()
            host, steps = 0.0, 20
            t0 = time.perf_counter()
            for _ in range(steps):
                h = time.perf_counter()
                ex.send(req, val, st)
                host += time.perf_counter() - h
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            res[name] = (val, st)
            row = {"host_enqueue_ms_per_step": round(host / steps * 1e3, 3),
                   "wall_ms_per_step": round(wall / steps * 1e3, 3)}
            if ex._engine is not None:  # native split of the enqueue cost, us per step
                p = ex._engine.host_profile()
                row.update({k.replace("_ns", "_us"): round(p[k] / p["sends"] / 1e3, 1)
                            for k in ("kernels_ns", "a2a_ns", "sync_ns", "total_ns")})
            out[f"chunks{chunks}_{name}"] = row
        ref = res["python_rccl"]
        same = all(torch.equal(v[0], ref[0]) and torch.equal(v[1], ref[1]) for v in res.values())
        out[f"chunks{chunks}_identical"] = bool(same)
        if not same:
            print(json.dumps(out))
            raise SystemExit("engine and python paths disagree")
    print(json.dumps(out))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Does an RCCL collective survive hipGraph capture here?  mode torch: torch's
own all_to_all_single captured; mode sx1 / sx2: the sorted exchange (1 / 2
chunks) captured.  One JSON line per run."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    mode = sys.argv[1]
    if mode == "sx1cs":  # the sorted exchange's collectives issued on the capturing stream itself
        os.environ["PTYPE_TUNE"] = "sx_comm_cs=1"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    if mode == "torch":
        x = torch.arange(1 << 20, dtype=torch.int64, device=dev)
        y = torch.empty_like(x)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            dist.all_to_all_single(y, x)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            dist.all_to_all_single(y, x)
        print("captured", file=sys.stderr, flush=True)
        y.zero_()
        g.replay()
        torch.cuda.synchronize()
        print(json.dumps({"mode": mode, "ok": bool(torch.equal(x, y))}))
    else:
        from ptype_amd.ops import batch as B
        from ptype_amd.ops.records import METHOD_CALC_MULTIPLY
        from ptype_amd.ops.table import RegistryTable, actor_keys
        from ptype_amd.parallel.exchange import ActorExchange

        n, M = 1 << 12, 1 << 16
        t = RegistryTable(2 * n, device=dev)
        ids = torch.arange(n)
        t.upsert(actor_keys(ids), torch.zeros(n, dtype=torch.int32), ids.to(torch.int32))
        t.enable_directory(n, affine_world=1)
        if mode == "eng":  # the epoch engine (direct delivery, wire v2 under capture)
            ex = ActorExchange(t, M, chunks=1, delivery="direct")
        else:
            ex = ActorExchange(t, M, chunks=1 if mode.startswith("sx1") else 2, delivery="mailbox",
                               mailbox_ordered=False)
        req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=1, device=dev)
        v = torch.empty(M, dtype=torch.int64, device=dev)
        s_ = torch.empty(M, dtype=torch.int32, device=dev)
        for _ in range(3):
            ex.send(req, v, s_)
        torch.cuda.synchronize()
        g = ex.capture(req, v, s_, allow_collectives=True)
        print("captured", file=sys.stderr, flush=True)
        v.zero_()
        g.replay()
        torch.cuda.synchronize()
        print(json.dumps({"mode": mode, "ok": bool(torch.equal(v, req.a0 * req.a1))}), flush=True)
        os._exit(0)  # (the teardown after a captured RCCL graph hung here once: skip it)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

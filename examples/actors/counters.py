#!/usr/bin/env python3
"""Stateful GPU actors across the node: every rank increments every counter actor.

    python examples/actors/counters.py                       # one GPU
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/actors/counters.py

Each process hosts ``--actors`` counter actors on its GPU (actor ``a`` lives on
rank ``a % world``).  Every rank sends ``CounterAdd(+1)`` to every actor of the
node ``--rounds`` times as one batched ``Send`` per round (GPU registry routing,
RCCL all-to-all epochs over xGMI), then each rank checks that its own actors
counted ``rounds * world`` and reads one back through the single-call path (the
persistent dispatcher, no kernel launch).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ptype_amd.ops.batch import MsgBatch  # noqa: E402
from ptype_amd.ops.records import METHOD_COUNTER_ADD, STATUS_OK  # noqa: E402
from ptype_amd.runtime import DeviceRuntime  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--actors", type=int, default=65536, help="actors per GPU")
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    rank = dist.get_rank() if world > 1 else 0
    rt = DeviceRuntime(dev, actors=a.actors, max_batch=a.actors * world)
    rt.place_local()
    n = rt.total_actors
    # every actor of the node, visited in a rank-specific order
    actors = torch.randperm(n, generator=torch.Generator().manual_seed(rank)).to(dev, torch.int32)
    batch = MsgBatch(actors, torch.ones(n, dtype=torch.int64, device=dev), None, None, METHOD_COUNTER_ADD)
    for _ in range(a.rounds):
        _, st = rt.send(None, batch)
        assert bool((st == STATUS_OK).all()), "undelivered messages"
    if world > 1:
        dist.barrier(device_ids=[local])
    torch.cuda.synchronize()
    ok = bool((rt.state == a.rounds * world).all())
    v, s = rt.call(METHOD_COUNTER_ADD, 0, 0)  # add 0: read mailbox 0 through the dispatcher
    print(f"rank {rank}: {rt.actors} actors, every counter == {a.rounds * world}: {ok}; "
          f"mailbox 0 via Call -> {v} (status {s})", flush=True)
    rt.close()
    if world > 1:
        dist.destroy_process_group()
    sys.exit(0 if ok and s == STATUS_OK else 1)


if __name__ == "__main__":
    main()

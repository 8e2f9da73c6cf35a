#!/usr/bin/env python3
"""Host time of Join -> NewClient -> Client.Send (utils/benchmarks.api_send) with
a cProfile of the Send loop: where a Client.Send's host microseconds go.
usage: python tools/api_send_profile.py [M]"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ptype_amd.utils import benchmarks as BM  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 8 << 20
    dev = torch.device("cuda", 0)
    pr = cProfile.Profile()
    orig = BM.timed

    def timed(step, steps, warmup, device, barrier=None):
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        pr.enable()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        pr.disable()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    BM.timed = timed
    try:
        out = BM.api_send(dev, [M], 131072, 20, 3)
    finally:
        BM.timed = orig
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumtime").print_stats(25)
    print(s.getvalue()[-6000:])
    print(out)


if __name__ == "__main__":
    main()

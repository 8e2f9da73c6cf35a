#!/usr/bin/env python3
"""Prime worker (reference example/optimus/worker/worker.go): serves
``Prime.Check(Args{Min, Max, Target})``.

The reference sleeps 250 ms per candidate to make the fan-out visible;
``PRIME_DELAY`` (seconds) overrides it.  With a ``gpu:`` section the method is
served by GPU actors (the per-candidate delay becomes the config's delay_us).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from _common import C, load_config, wait_for_signal  # noqa: E402

from ptype_amd.models import optimus  # noqa: E402


def main():
    cfg = load_config()
    server = C.Server()
    if not cfg.has_gpu:
        server.Register(optimus.Prime(delay=float(os.environ.get("PRIME_DELAY", "0.25"))))
        # listen BEFORE registering: the reference registers first (worker.go Join,
        # then ListenAndServe), so a mesh client that dials the new node at once can
        # be refused -- the coordinator's initial connect then fails (rpc.go:278-280)
        server.Listen(cfg.port)
    c = C.Join(C.background(), cfg)
    if cfg.has_gpu:  # device methods need the joined runtime; listen once they are bound
        c.runtime.serve(server, optimus.SERVICE, optimus.DEVICE_METHODS)
        server.Listen(cfg.port)
    print(f"worker: services {c.Registry.Services(C.background())}", flush=True)
    try:
        wait_for_signal()
    finally:
        server.Close()
        c.Close()


if __name__ == "__main__":
    main()

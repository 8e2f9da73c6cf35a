#!/usr/bin/env python3
"""Calculator server (reference example/calculator/server/server.go).

Registers ``Calculator`` with the net/rpc server, joins the cluster, prints the
services it sees and serves ``:port`` until stopped.  With a ``gpu:`` section in
the config (calculator_server_gpu.yaml) ``Calculator.Multiply`` is served by a
GPU actor through the persistent dispatcher instead of the host receiver; the
wire protocol seen by clients is identical.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from _common import C, load_config, wait_for_signal  # noqa: E402

from ptype_amd.models import calculator  # noqa: E402


def main():
    cfg = load_config()
    server = C.Server()
    if not cfg.has_gpu:
        server.Register(calculator.Calculator())
        server.Listen(cfg.port)  # before registering, so a client that sees the node can dial it
    c = C.Join(C.background(), cfg)
    if cfg.has_gpu:  # device methods need the joined runtime; listen once they are bound
        calculator.serve_device(c.runtime, server)
        server.Listen(cfg.port)
    print(f"server: services {c.Registry.Services(C.background())}", flush=True)
    try:
        wait_for_signal()
    finally:
        server.Close()
        c.Close()


if __name__ == "__main__":
    main()

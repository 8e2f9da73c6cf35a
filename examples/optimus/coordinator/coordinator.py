#!/usr/bin/env python3
"""Optimus coordinator (reference example/optimus/coordinator/coordinator.go).

Joins the cluster, opens a full-mesh client to ``prime_worker`` and serves
``POST /test`` (form ``target=<int>``) on :8082: the range [2, target) is split
into 10-wide chunks, fanned out concurrently with ``Client.Go`` and the first
reply that is not ``target`` wins.  ``COORDINATOR_HTTP_PORT`` overrides 8082.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from _common import C, load_config, wait_for_signal  # noqa: E402

from ptype_amd.models import optimus  # noqa: E402


def main():
    cfg = load_config()
    c = C.Join(C.background(), cfg)
    worker = c.NewClient("prime_worker", C.ConnConfig(max_connections=0))  # mesh: every replica
    coord = optimus.Coordinator(lambda t: optimus.check_host(worker, t),
                                port=int(os.environ.get("COORDINATOR_HTTP_PORT", "8082")), host="0.0.0.0")
    print(f"coordinator: serving /test on :{coord.port}", flush=True)
    try:
        wait_for_signal()
    finally:
        coord.close()
        worker.Close()
        c.Close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Calculator client (reference example/calculator/client/client.go): join,
list services, give the server's HTTP listener a moment, then
``Calculator.Multiply(Args{7, 8})``."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from _common import C, load_config  # noqa: E402

from ptype_amd.models.calculator import Args  # noqa: E402


def main():
    cfg = load_config()
    c = C.Join(C.background(), cfg)
    try:
        print(f"client: services {c.Registry.Services(C.background())}", flush=True)
        time.sleep(0.5)  # the server's listener comes up after its member
        client = c.NewClient("calculator", None)
        try:
            args = Args(7, 8)
            reply = client.Call("Calculator.Multiply", args)
            print(f"client: {args.A}*{args.B}={reply}", flush=True)
        finally:
            client.Close()
    finally:
        c.Close()


if __name__ == "__main__":
    main()

"""Shared helpers of the example programs: load ``CONFIG``, keep a server alive
until SIGINT/SIGTERM, and make the repo importable when run from a checkout."""
from __future__ import annotations

import os
import signal
import sys
import threading

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from ptype_amd import cluster as C  # noqa: E402


def load_config():
    """``cluster.ConfigFromFile(os.Getenv("CONFIG"))`` -- the reference's only knob."""
    path = os.environ.get("CONFIG")
    if not path:
        sys.exit("CONFIG must name the service YAML")
    return C.ConfigFromFile(path)


def wait_for_signal() -> None:
    """Block like ``http.ListenAndServe`` until the process is told to stop."""
    done = threading.Event()
    for s in (signal.SIGINT, signal.SIGTERM):
        signal.signal(s, lambda *_: done.set())
    done.wait()

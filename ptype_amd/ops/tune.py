"""The data plane's path switches (csrc/hip/tune.hpp holds the native ones).

One environment variable, ``PTYPE_TUNE="key=value,key=value"``, or the config's
``gpu: tune:`` map (``set``), selects between implementations that are kept on
purpose: the default is the measured-faster one, the other a reference a GPU
test compares against or a path for a case the default does not cover.  Python
keys (read when an exchange is built or per Send):

  key              default  meaning
  engine           1        native epoch engine on a GPU (0: the Python/torch pipeline)
  wire             3        wire format of the epoch engine's all-to-alls (2: v2)
  adaptive_c       1        agreed slot capacity (0 off, 2 also at world 1 with collectives)
  skew_room        4        epoch-engine buffers: x the uniform share per peer
  sorted_room      2.5      sorted-exchange buffers: x the uniform share per peer
  direct           -1       direct completion of self-directed messages (-1: world 1 only)
  sorted_exchange  1        N > 1 mailbox delivery through the sorted exchange
  device_pump      1        device-counted pump epochs (0: a host round trip per epoch)
  pump_graph       1        world-1 pump groups replayed from a hipGraph
  auto_arrival     1        world-1 mailbox Sends without ordered methods, up to 2 Mi
                            messages: arrival rings (0: the actor-sharded sort)

The native keys are listed in csrc/hip/tune.hpp; ``set`` forwards them.
"""
from __future__ import annotations

import os

_PY_DEFAULTS = {"engine": 1, "wire": 3, "adaptive_c": 1, "skew_room": 4.0, "sorted_room": 2.5, "direct": -1,
                "sorted_exchange": 1, "device_pump": 1, "pump_graph": 1,
                "auto_arrival": 1}
_overrides: dict[str, str] = {}


def _parse(spec: str) -> dict[str, str]:
    out = {}
    for item in spec.split(","):
        if "=" in item:
            k, v = item.split("=", 1)
            out[k.strip()] = v.strip()
    return out


def get(key: str):
    """The value in force for a Python key (environment, then ``set`` overrides)."""
    if key not in _PY_DEFAULTS:
        raise KeyError(f"unknown tune key {key!r}")
    d = _PY_DEFAULTS[key]
    vals = _parse(os.environ.get("PTYPE_TUNE", ""))
    vals.update(_overrides)
    v = vals.get(key)
    if v is None:
        return d
    return type(d)(float(v)) if isinstance(d, int) else type(d)(v)


def set(spec) -> None:  # noqa: A001 - the config's verb
    """Apply ``spec`` (a dict or "k=v,k=v"): Python keys here, native keys in the
    device runtime (``_hip.set_tune``).  Unknown keys raise ``KeyError``."""
    items = spec if isinstance(spec, dict) else _parse(str(spec))
    native = {}
    for k, v in items.items():
        if k in _PY_DEFAULTS:
            _overrides[k] = str(v)
        else:
            native[k] = str(v)
    if native:
        from . import hip

        if not hip().set_tune(",".join(f"{k}={v}" for k, v in native.items())):
            raise KeyError(f"unknown tune key(s): {sorted(native)}")

"""Reference workloads: the calculator and optimus examples (host + GPU paths)."""
from . import calculator, optimus  # noqa: F401

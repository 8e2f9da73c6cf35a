"""The engine's default cross-stream hand-off under the profiler.

A rocprofv3 counter pass over the RCCL path once hung with stream wait-value
hand-offs (csrc/hip/engine.hpp, handoff()); events are the default since.  This
runs the default hand-off on the RCCL path (--force-dist: process group up, both
all-to-alls through ncclAllToAll) under `rocprofv3 --kernel-trace` to completion,
and checks that the trace saw the route / dispatch kernels (the sorted
exchange's sort / drain kernels for mailbox delivery) and RCCL's own."""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT, free_port


@pytest.mark.gpu
def test_default_handoff_under_rocprofv3_kernel_trace(tmp_path):
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        pytest.skip("rocprofv3 not installed")
    env = dict(os.environ, TMPDIR="/tmp", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()),
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("PTYPE_TUNE", None)  # the default hand-off
    out = tmp_path / "trace"
    cmd = [prof, "--kernel-trace", "--stats", "-d", str(out), "-o", "run", "--output-format", "csv", "--",
           sys.executable, "bench.py", "--force-dist", "--steps", "3", "--warmup", "1", "--rtt-calls", "0",
           "--msgs-per-gpu", str(1 << 20), "--no-secondary"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    assert any(ln.startswith("{") for ln in p.stdout.splitlines()), p.stdout[-2000:]
    stats = [os.path.join(d, f) for d, _, fs in os.walk(out) for f in fs if f.endswith("kernel_stats.csv")]
    assert stats, list(os.walk(out))
    text = open(stats[0]).read()
    # mailbox delivery at N > 1 is the sorted exchange (sender-side sort, receiver drain)
    # (sender: count + scatter, or the one-pass reserving sort for rank-only batches)
    assert ("dispatch" in text and "route" in text) or \
        (("sx_scatter" in text or "sx_onesweep" in text) and "sx_drain" in text), text[:2000]
    assert "nccl" in text.lower() or "rccl" in text.lower() or "alltoall" in text.lower(), text[:2000]

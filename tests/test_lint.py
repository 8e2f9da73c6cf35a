"""The lint step passes (reference CI: gofmt + golangci-lint/errcheck before the
tests, Makefile:4-6, .travis.yml:9-10): format, unused imports, the host control
plane under -Wall -Wextra -Werror, and -- where hipcc exists -- errcheck on every
HIP call of the device runtime (tools/lint.py --native)."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT


@pytest.mark.timeout(600)
def test_lint_clean():
    args = [sys.executable, os.path.join(ROOT, "tools", "lint.py")]
    if os.path.exists(os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")):
        args.append("--native")
    p = subprocess.run(args, cwd=ROOT, capture_output=True, text=True, timeout=580)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]

"""CMakeLists.txt (the production build of _core and _hip, equivalent to
ptype_amd/_build.py) configures for gfx950 only.  The full build is exercised
by hand / CI (`cmake --build`); configuring is cheap enough for every run."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("cmake") is None or not os.path.exists("/opt/rocm/lib/llvm/bin/clang++"),
                    reason="cmake / ROCm clang not available")
def test_cmake_configures_for_gfx950(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run(["cmake", "-S", ROOT, "-B", str(tmp_path / "b"), "-DCMAKE_PREFIX_PATH=/opt/rocm",
                        "-DCMAKE_HIP_COMPILER=/opt/rocm/lib/llvm/bin/clang++",
                        f"-DPTYPE_OUTPUT_DIR={tmp_path / 'out'}"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    cache = (tmp_path / "b" / "CMakeCache.txt").read_text()
    assert "CMAKE_HIP_ARCHITECTURES:STRING=gfx950" in cache

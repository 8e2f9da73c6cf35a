"""The example programs run end to end as separate processes, like the
reference's `run` scripts (fixed ports from the reference configs)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, script, env=None, timeout=150):
    ex = tmp_path / "examples"
    shutil.copytree(os.path.join(ROOT, "examples"), ex)
    e = dict(os.environ, PYTHONPATH=ROOT, **(env or {}))
    return subprocess.run([str(ex / script)], env=e, capture_output=True, text=True, timeout=timeout)


def test_calculator_example_processes(tmp_path):
    r = _run(tmp_path, "calculator/run")
    assert r.returncode == 0, r.stderr[-2000:]
    assert "client: 7*8=56" in r.stdout
    assert "server: services" in r.stdout and "calculator_client" in r.stdout


def test_optimus_example_processes(tmp_path):
    r = _run(tmp_path, "optimus/run", {"PRIME_DELAY": "0", "TARGET": "221", "COORDINATOR_HTTP_PORT": "18082"})
    assert r.returncode == 0, r.stderr[-2000:]
    assert "target=221 -> 13" in r.stdout


@pytest.mark.gpu
def test_calculator_example_gpu_server(tmp_path):
    r = _run(tmp_path, "calculator/run", {"GPU": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    assert "client: 7*8=56" in r.stdout


@pytest.mark.gpu
def test_gpu_counter_actors_example():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples/actors/counters.py"), "--actors", "4096"],
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert "every counter == 3: True" in r.stdout

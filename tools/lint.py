#!/usr/bin/env python3
"""Lint step (the reference's `make lint`: gofmt + golangci-lint with errcheck,
Makefile:4-6, .golangci.yml:1-3, run by CI before the tests, .travis.yml:9-10).

No third-party linters ship in this image, so the checks are built from the
toolchain and the standard library:

* format (the gofmt analogue), every source file: no tabs, no trailing
  whitespace, lines <= 160 columns, a final newline;
* Python: the file compiles, and no import is unused (an AST pass; a name a
  module re-exports through ``__all__`` or marks ``# noqa`` counts as used);
* C++ (host control plane): ``g++ -fsyntax-only -Wall -Wextra -Werror``;
* HIP (``--native``): ``hipcc -fsyntax-only -Wall -Werror=unused-value
  -Werror=unused-result`` -- a ``hipError_t`` is ``[[nodiscard]]``, so this is
  errcheck for the device runtime: every ignored HIP error must be a visible
  ``(void)`` cast.

Exit status 1 with one line per finding.  ``python tools/lint.py [--native]``.
"""
from __future__ import annotations

import argparse
import ast
import glob
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAX_COL = 160  # the repo's style is ~120; 160 flags only runaway lines
PY_GLOBS = ["ptype_amd/**/*.py", "tests/**/*.py", "tools/**/*.py", "examples/**/*.py", "bench.py",
            "__graft_entry__.py"]
CXX_GLOBS = ["ptype_amd/csrc/**/*.cpp", "ptype_amd/csrc/**/*.hpp", "ptype_amd/csrc/**/*.hip", "tests/native/*.cpp",
             "tools/*.hip"]


def files(globs):
    out = []
    for g in globs:
        out += glob.glob(os.path.join(ROOT, g), recursive=True)
    return sorted(set(out))


def check_format(path):
    out = []
    with open(path, encoding="utf-8") as f:
        text = f.read()
    if text and not text.endswith("\n"):
        out.append(f"{path}: no newline at end of file")
    for i, line in enumerate(text.split("\n"), 1):
        if "\t" in line:
            out.append(f"{path}:{i}: tab")
        if line.rstrip() != line:
            out.append(f"{path}:{i}: trailing whitespace")
        if len(line) > MAX_COL:
            out.append(f"{path}:{i}: {len(line)} columns (max {MAX_COL})")
    return out


class _Names(ast.NodeVisitor):
    def __init__(self):
        self.used = set()

    def visit_Name(self, node):
        self.used.add(node.id)

    def visit_Attribute(self, node):
        base = node
        while isinstance(base, ast.Attribute):
            base = base.value
        if isinstance(base, ast.Name):
            self.used.add(base.id)
        self.generic_visit(node)


def check_python(path):
    with open(path, encoding="utf-8") as f:
        src = f.read()
    try:
        tree = ast.parse(src, path)
        compile(src, path, "exec")
    except SyntaxError as e:
        return [f"{path}:{e.lineno}: syntax error: {e.msg}"]
    lines = src.split("\n")
    names = _Names()
    names.visit(tree)
    exported = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "__all__" for t in node.targets):
            if isinstance(node.value, (ast.List, ast.Tuple)):
                exported |= {e.value for e in node.value.elts if isinstance(e, ast.Constant)}
    # names used only inside string annotations count as used
    for node in ast.walk(tree):
        if isinstance(node, ast.Constant) and isinstance(node.value, str):
            for tok in node.value.replace("[", " ").replace("]", " ").replace("|", " ").replace(",", " ").split():
                names.used.add(tok.split(".")[0])
    out = []
    is_init = os.path.basename(path) == "__init__.py"
    for node in ast.walk(tree):
        if not isinstance(node, (ast.Import, ast.ImportFrom)):
            continue
        if isinstance(node, ast.ImportFrom) and node.module == "__future__":
            continue
        stmt = "\n".join(lines[node.lineno - 1:(node.end_lineno or node.lineno)])
        if "noqa" in stmt or is_init:
            continue
        for a in node.names:
            bound = (a.asname or a.name).split(".")[0]
            if a.name == "*" or bound in names.used or bound in exported:
                continue
            out.append(f"{path}:{node.lineno}: unused import {a.name}")
    return out


def _pybind_include():
    import pybind11

    return pybind11.get_include()


def check_cxx_host():
    core = os.path.join(ROOT, "ptype_amd", "csrc", "core")
    flags = ["-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-I" + core, "-I" + _pybind_include(),
             "-I" + sysconfig.get_paths()["include"]]
    srcs = sorted(glob.glob(os.path.join(core, "*.cpp")))

    def one(s):
        p = subprocess.run(["g++"] + flags + [s], capture_output=True, text=True)
        return [f"{s}: {ln}" for ln in p.stderr.splitlines() if "error" in ln or "warning" in ln] if p.returncode else []

    with ThreadPoolExecutor(8) as ex:
        return [x for r in ex.map(one, srcs) for x in r]


def check_hip():
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    hipcc = os.path.join(rocm, "bin", "hipcc")
    if not os.path.exists(hipcc):
        return ["hipcc not found: HIP sources not checked"]
    hipdir = os.path.join(ROOT, "ptype_amd", "csrc", "hip")
    flags = ["-x", "hip", "-std=c++17", "-fsyntax-only", "--offload-arch=gfx950", "-Wall", "-Werror=unused-value",
             "-Werror=unused-result", "-Wno-unused-command-line-argument", "-I" + hipdir,
             "-I" + os.path.join(ROOT, "ptype_amd", "csrc", "core"), "-I" + _pybind_include(),
             "-I" + sysconfig.get_paths()["include"]]
    srcs = sorted(glob.glob(os.path.join(hipdir, "*.hip")) + glob.glob(os.path.join(hipdir, "*.cpp")))

    def one(s):
        p = subprocess.run([hipcc] + flags + [s], capture_output=True, text=True)
        return [f"{s}: {ln}" for ln in p.stderr.splitlines() if "error" in ln] if p.returncode else []

    with ThreadPoolExecutor(8) as ex:
        return [x for r in ex.map(one, srcs) for x in r]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--native", action="store_true", help="also check the HIP sources with hipcc (errcheck)")
    ap.add_argument("--no-cxx", action="store_true", help="skip the g++ pass over the host control plane")
    a = ap.parse_args(argv)
    findings = []
    py = files(PY_GLOBS)
    for p in py:
        findings += check_format(p)
        findings += check_python(p)
    for p in files(CXX_GLOBS):
        findings += check_format(p)
    if not a.no_cxx:
        findings += check_cxx_host()
    if a.native:
        findings += check_hip()
    for f in findings:
        print(os.path.relpath(f, ROOT) if f.startswith(ROOT) else f)
    print(f"lint: {len(findings)} finding(s) in {len(py)} Python and {len(files(CXX_GLOBS))} C++/HIP files",
          file=sys.stderr)
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main())

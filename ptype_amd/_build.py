"""Native build driver for ptype_amd (no setuptools, no JIT cache).

Builds two in-tree extension modules:

* ``ptype_amd/_core*.so`` -- host-only C++17 control plane (config/YAML, MVCC KV,
  leases, watch, Raft, TCP transport, registry, KV store, balancer, Go net/rpc
  gob codec).  Compiled with g++; no HIP dependency so it can be built with
  host sanitizers (``PTYPE_SANITIZE=thread|address``).
* ``ptype_amd/_hip*.so`` -- HIP/CDNA4 device runtime (gfx950 only): HBM mailbox
  rings, GPU registry hash table, route/dispatch/complete kernels, persistent
  dispatcher, snapshot pack kernels.  Compiled with hipcc ``--offload-arch=gfx950``.

Incremental: an object is rebuilt when its source or any header under ``csrc``
is newer than the object.  Objects live in ``build/`` (git-ignored).
"""
from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = "gfx950"
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _pybind_include() -> str:
    import pybind11

    return pybind11.get_include()


def _py_include() -> str:
    return sysconfig.get_paths()["include"]


def _newest_header(d: str) -> float:
    t = 0.0
    for h in glob.glob(os.path.join(d, "**", "*.hpp"), recursive=True) + glob.glob(
        os.path.join(d, "**", "*.h"), recursive=True
    ):
        t = max(t, os.path.getmtime(h))
    return t


def _run(cmd: list[str], log: str | None = None) -> None:
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if p.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + p.stdout)
    if log:
        with open(log, "w") as f:
            f.write(p.stdout)


def _compile_logged(jobs, max_workers):
    with ThreadPoolExecutor(max_workers=max_workers) as ex:
        list(ex.map(lambda j: _run(j[0], j[1]), jobs))


def kernel_resources() -> dict:
    """Per-kernel VGPRs / scratch / occupancy from the last hipcc compile of each
    object (``-Rpass-analysis=kernel-resource-usage`` remarks, kept next to the
    objects).  A kernel with scratch > 0 is a performance bug on gfx950."""
    out = {}
    for res in glob.glob(os.path.join(ROOT, "build", "hip", "*.res")):
        cur = None
        for line in open(res):
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                cur = out.setdefault(m.group(1), {})
                continue
            m = re.search(r"(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
            if m and cur is not None:
                cur[m.group(1).split(" ")[0]] = int(m.group(2))
    return out


def _compile_all(jobs, max_workers):
    with ThreadPoolExecutor(max_workers=max_workers) as ex:
        list(ex.map(_run, jobs))


def _variant_dir(name: str, sanitize: str | None) -> str:
    d = os.path.join(ROOT, "build", name + (("-" + sanitize) if sanitize else ""))
    os.makedirs(d, exist_ok=True)
    return d


def build_core(verbose: bool = False, sanitize: str | None = None, out: str | None = None) -> str:
    """Build the host-only control-plane module ``_core``."""
    sanitize = sanitize or os.environ.get("PTYPE_SANITIZE") or None
    srcs = sorted(glob.glob(os.path.join(CSRC, "core", "*.cpp")))
    objdir = _variant_dir("core", sanitize)
    hdr_t = _newest_header(os.path.join(CSRC, "core"))
    cxx = os.environ.get("CXX", "g++")
    flags = [
        "-std=c++17", "-O2", "-g1", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
        "-pthread", "-I" + os.path.join(CSRC, "core"), "-I" + _pybind_include(), "-I" + _py_include(),
    ]
    if sanitize:
        flags += ["-fsanitize=" + sanitize, "-fno-omit-frame-pointer", "-O1"]
    jobs, objs = [], []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_t):
            jobs.append([cxx] + flags + ["-c", s, "-o", o])
    _compile_all(jobs, 8)
    target = out or os.path.join(PKG, "_core" + EXT)
    if jobs or not os.path.exists(target) or os.path.getmtime(target) < max(os.path.getmtime(o) for o in objs):
        link = [cxx, "-shared", "-pthread", "-o", target] + objs
        if sanitize:
            link += ["-fsanitize=" + sanitize]
        _run(link)
    if verbose:
        print("built", target, "(%d objects recompiled)" % len(jobs))
    return target


def _torch_lib_dir() -> str | None:
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            d = os.path.join(os.path.dirname(spec.origin), "lib")
            if os.path.exists(os.path.join(d, "libamdhip64.so")):
                return d
    except Exception:
        pass
    return None


def build_hip(verbose: bool = False) -> str:
    """Build the gfx950 device-runtime module ``_hip`` with hipcc.

    The module links the HIP runtime that ships inside torch (SONAME
    libamdhip64.so.7) when present, so a process that imports torch first has
    exactly ONE HIP runtime (torch's) -- tensors, streams and our kernels share it.
    """
    srcs = sorted(glob.glob(os.path.join(CSRC, "hip", "*.hip")) + glob.glob(os.path.join(CSRC, "hip", "*.cpp")))
    objdir = _variant_dir("hip", None)
    hdr_t = max(_newest_header(os.path.join(CSRC, "hip")), _newest_header(os.path.join(CSRC, "core")))
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    flags = [
        "-std=c++17", "-O3", "-fPIC", "-fvisibility=hidden", "--offload-arch=" + ARCH,
        "-Wno-unused-result", "-munsafe-fp-atomics",
        "-I" + os.path.join(CSRC, "hip"), "-I" + os.path.join(CSRC, "core"),
        "-I" + _pybind_include(), "-I" + _py_include(),
    ]
    jobs, objs = [], []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        lang = ["-x", "hip"]
        # (a source may include another .hip: mailbox_sort_fused_other.hip)
        inc = [os.path.join(os.path.dirname(s), m) for m in re.findall(r'#include "([^"]+\.hip)"', open(s).read())]
        src_t = max([os.path.getmtime(s)] + [os.path.getmtime(i) for i in inc if os.path.exists(i)])
        if not os.path.exists(o) or os.path.getmtime(o) < max(src_t, hdr_t):
            jobs.append(([hipcc] + lang + flags + ["-Rpass-analysis=kernel-resource-usage", "-c", s, "-o", o],
                         o[:-2] + ".res"))
    _compile_logged(jobs, 8)
    target = os.path.join(PKG, "_hip" + EXT)
    tl = _torch_lib_dir()
    if jobs or not os.path.exists(target) or os.path.getmtime(target) < max(os.path.getmtime(o) for o in objs):
        # libhsa-runtime64 (soname .so.1) for hsa_amd_pointer_info: resolved through the
        # RUNPATH to the runtime torch's HIP already loaded
        link = [hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", target] + objs + [
            "-L" + os.path.join(ROCM, "lib"), "-lhsa-runtime64"]
        if tl:
            # bind to torch's runtime first (same SONAME as /opt/rocm's)
            link += ["-Wl,-rpath," + tl]
        _run(link)
    if verbose:
        print("built", target, "(%d objects recompiled)" % len(jobs))
    return target


SANITIZERS = {
    "thread": ["-fsanitize=thread"],
    "address": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
}


def build_native_test(sanitize: str = "thread", verbose: bool = False) -> str:
    """Build ``tests/native/core_stress`` -- the host control plane without
    Python, under a sanitizer (the reference runs ``go test -race``).

    The sanitizer runtime must own the process, which a Python extension cannot
    give it, so the control-plane sources are linked into a native program.
    Objects go to ``build/native-<sanitize>/``; returns the executable path.
    """
    if sanitize not in SANITIZERS:
        raise ValueError(f"sanitize must be one of {sorted(SANITIZERS)}")
    srcs = [s for s in sorted(glob.glob(os.path.join(CSRC, "core", "*.cpp"))) if not s.endswith("bindings.cpp")]
    srcs.append(os.path.join(ROOT, "tests", "native", "core_stress.cpp"))
    objdir = _variant_dir("native", sanitize)
    hdr_t = _newest_header(os.path.join(CSRC, "core"))
    # LLVM's sanitizer runtimes (ROCm's clang): gcc 11's libtsan lacks the
    # pthread_cond_clockwait interceptor that libstdc++'s wait_for uses, which
    # shows up as false "double lock" / race reports on every condition variable
    clang = os.path.join(ROCM, "lib", "llvm", "bin", "clang++")
    cxx = os.environ.get("PTYPE_SAN_CXX") or (clang if os.path.exists(clang) else "g++")
    flags = ["-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", "-Wall", "-Wno-unused-function",
             "-I" + os.path.join(CSRC, "core")] + SANITIZERS[sanitize]
    jobs, objs = [], []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_t):
            jobs.append([cxx] + flags + ["-c", s, "-o", o])
    _compile_all(jobs, 8)
    target = os.path.join(objdir, "core_stress")
    if jobs or not os.path.exists(target) or os.path.getmtime(target) < max(os.path.getmtime(o) for o in objs):
        _run([cxx, "-pthread", "-o", target] + objs + SANITIZERS[sanitize])
    if verbose:
        print("built", target, "(%d objects recompiled)" % len(jobs))
    return target


def build_all(verbose: bool = False) -> None:
    # the two modules share nothing: the host objects compile while hipcc works
    # through the device runtime (its longest object sets the wall time)
    with ThreadPoolExecutor(max_workers=2) as ex:
        for f in [ex.submit(build_core, verbose), ex.submit(build_hip, verbose)]:
            f.result()


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what == "core":
        build_core(True)
    elif what == "hip":
        build_hip(True)
    elif what.startswith("native-"):
        build_native_test(what.split("-", 1)[1], True)
    else:
        build_all(True)

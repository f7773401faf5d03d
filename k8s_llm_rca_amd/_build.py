"""In-tree build of the native pieces (no pip install, no JIT cache).

* ``_graphcore.<abi>.so`` - C++ host graph operators (pybind11, g++ -O3).
* ``libk8srca_hip.so``    - every HIP/CDNA4 kernel, compiled for gfx950 only with
  hipcc and exposed through a plain C ABI (``csrc/kernels/*.hip``).  It is
  loaded with ctypes *after* ``import torch`` so it binds to the same
  ``libamdhip64.so.7`` runtime torch already loaded (same SONAME).

Both land next to this file so a ``gpurun`` snapshot carries them to the GPU
box.  Rebuilds are incremental on source mtime.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig
from typing import List

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
ARCH = os.environ.get("K8SRCA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _newer(target: str, sources: List[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: %s\n%s\n%s" % (" ".join(cmd), r.stdout[-4000:], r.stderr[-8000:]))


def graphcore_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_graphcore" + suffix)


def build_graphcore(force: bool = False) -> str:
    import pybind11

    src = os.path.join(CSRC, "graph", "graphcore.cpp")
    hdr = os.path.join(CSRC, "graph", "graphcore_core.h")
    out = graphcore_path()
    if force or _newer(out, [src, hdr]):
        inc = sysconfig.get_paths()["include"]
        tmp = out + ".tmp"
        _run(["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
              "-I", pybind11.get_include(), "-I", inc, src, "-o", tmp])
        os.replace(tmp, out)
    return out


def hip_lib_path() -> str:
    return os.path.join(PKG, "libk8srca_hip.so")


def hip_sources() -> List[str]:
    return sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))


def build_hip(force: bool = False, jobs: int = 8) -> str:
    """Compile every kernel TU to an object (in parallel) and link one .so."""
    srcs = hip_sources()
    hdrs = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    out = hip_lib_path()
    objdir = os.path.join(PKG, "csrc", "build")
    os.makedirs(objdir, exist_ok=True)
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-ffp-contract=fast", "-I", os.path.join(CSRC, "kernels")]
    procs = []
    objs = []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + hdrs):
            procs.append((s, subprocess.Popen([HIPCC, *flags, "-c", s, "-o", o],
                                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
            if len(procs) >= jobs:
                _drain(procs)
    _drain(procs)
    if force or _newer(out, objs):
        tmp = out + ".tmp"
        # -lhipblaslt resolves (SONAME libhipblaslt.so.1) to the copy torch already
        # mapped when the library is loaded after `import torch`: one hipBLASLt per process
        # -z defs: an unresolved symbol (e.g. a kernel launch stub the host pass
        # dropped) fails the build here, not the first dlopen on the GPU box
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-L/opt/rocm/lib", "-lhipblaslt",
              "-Wl,-z,defs", "-o", tmp])
        os.replace(tmp, out)
    return out


def _drain(procs):
    errs = []
    while procs:
        s, p = procs.pop(0)
        so, se = p.communicate()
        if p.returncode != 0:
            errs.append(f"{s}:\n{se[-6000:]}")
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))


def build_all(force: bool = False) -> None:
    build_graphcore(force)
    build_hip(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("built", graphcore_path(), hip_lib_path())


def build_graphcore_sanitized(out_dir: str) -> str:
    """Standalone test driver of the graph core under ASan + UBSan (host only;
    SURVEY.md §5.2).  Returns the executable path."""
    src = os.path.join(CSRC, "graph", "graphcore_test.cpp")
    exe = os.path.join(out_dir, "graphcore_test_asan")
    _run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
          "-fno-sanitize-recover=undefined", "-I", os.path.join(CSRC, "graph"), src, "-o", exe])
    return exe

"""In-tree build of the native pieces (no pip install, no JIT cache).

* ``_graphcore.<abi>.so`` - C++ host graph operators (pybind11, g++ -O3).
* ``libk8srca_hip.so``    - every HIP/CDNA4 kernel, compiled for gfx950 only with
  hipcc and exposed through a plain C ABI (``csrc/kernels/*.hip``).  It is
  loaded with ctypes *after* ``import torch`` so it binds to the same
  ``libamdhip64.so.7`` runtime torch already loaded (same SONAME).

Both land next to this file so a ``gpurun`` snapshot carries them to the GPU
box.  Rebuilds are incremental on CONTENT, not mtime: each
output has a ``.sha`` sidecar holding the SHA-256 of its compiler command,
sources and headers, and anything whose digest differs is rebuilt -- a snapshot
whose objects are newer than edited sources still recompiles.  Every compile
is logged (``k8s_llm_rca_amd.build``) and listed in :data:`LAST_BUILD`.
"""
from __future__ import annotations

import glob
import hashlib
import logging
import os
import subprocess
import sys
import sysconfig
from typing import List

from .knobs import KNOBS

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
ARCH = KNOBS.offload_arch
HIPCC = KNOBS.hipcc
log = logging.getLogger("k8s_llm_rca_amd.build")
# outputs (re)built by the last build_* call of this process
LAST_BUILD: List[str] = []


def _digest(cmd: List[str], inputs: List[str]) -> str:
    h = hashlib.sha256("\0".join(cmd).encode())
    for p in sorted(inputs):
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _stale(target: str, digest: str) -> bool:
    """True unless ``target`` exists and was built from exactly ``digest``."""
    try:
        with open(target + ".sha") as f:
            return not os.path.exists(target) or f.read().strip() != digest
    except OSError:
        return True


def _stamp(target: str, digest: str) -> None:
    with open(target + ".sha", "w") as f:
        f.write(digest + "\n")
    LAST_BUILD.append(os.path.relpath(target, PKG))
    log.info("built %s", os.path.relpath(target, PKG))


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
    inc = sysconfig.get_paths()["include"]
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
           "-I", pybind11.get_include(), "-I", inc, src]
    dg = _digest(cmd, [src, hdr])
    if force or _stale(out, dg):
        tmp = out + ".tmp"
        _run(cmd + ["-o", tmp])
        os.replace(tmp, out)
        _stamp(out, dg)
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
        dg = _digest([HIPCC, *flags, "-c"], [s] + hdrs)
        if force or _stale(o, dg):
            procs.append(((s, o, dg), subprocess.Popen([HIPCC, *flags, "-c", s, "-o", o],
                                                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
            if len(procs) >= jobs:
                _drain(procs)
    _drain(procs)
    # -lhipblaslt resolves (SONAME libhipblaslt.so.1) to the copy torch already
    # mapped when the library is loaded after `import torch`: one hipBLASLt per process
    # -z defs: an unresolved symbol (e.g. a kernel launch stub the host pass
    # dropped) fails the build here, not the first dlopen on the GPU box
    link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-L/opt/rocm/lib", "-lhipblaslt",
            "-Wl,-z,defs"]
    dg = _digest(link, objs)
    if force or _stale(out, dg):
        tmp = out + ".tmp"
        _run(link + ["-o", tmp])
        os.replace(tmp, out)
        _stamp(out, dg)
    return out


def _drain(procs):
    errs = []
    while procs:
        (s, o, dg), p = procs.pop(0)
        so, se = p.communicate()
        if p.returncode != 0:
            errs.append(f"{s}:\n{se[-6000:]}")
        else:
            _stamp(o, dg)
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))


def build_all(force: bool = False) -> List[str]:
    """Build what is stale (everything with ``force``); returns the outputs built."""
    del LAST_BUILD[:]
    build_graphcore(force)
    build_hip(force)
    return list(LAST_BUILD)


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

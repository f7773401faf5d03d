"""In-tree build hygiene: rebuilds follow source CONTENT,
not mtime, and the driver's ``build()`` always compiles."""
import os
import shutil
import subprocess

import pytest

from k8s_llm_rca_amd import _build

KERNEL = """#include <hip/hip_runtime.h>
__global__ void k_add(float* x, float v) { x[threadIdx.x] += v; }
extern "C" int k_probe(float* x, hipStream_t s) {
  hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, s, x, %s);
  return (int)hipGetLastError();
}
"""


def _tree(tmp_path, monkeypatch):
    pkg = tmp_path / "pkg"
    (pkg / "csrc" / "kernels").mkdir(parents=True)
    (pkg / "csrc" / "kernels" / "probe.hip").write_text(KERNEL % "1.0f")
    (pkg / "csrc" / "kernels" / "probe.h").write_text("// header\n")
    monkeypatch.setattr(_build, "PKG", str(pkg))
    monkeypatch.setattr(_build, "CSRC", str(pkg / "csrc"))
    return pkg


@pytest.mark.skipif(shutil.which(_build.HIPCC) is None and not os.path.exists(_build.HIPCC), reason="no hipcc")
def test_backdated_kernel_edit_recompiles(tmp_path, monkeypatch):
    pkg = _tree(tmp_path, monkeypatch)
    src = pkg / "csrc" / "kernels" / "probe.hip"
    del _build.LAST_BUILD[:]
    _build.build_hip(jobs=2)
    assert _build.LAST_BUILD == ["csrc/build/probe.hip.o", "libk8srca_hip.so"]
    # nothing changed: nothing is compiled
    del _build.LAST_BUILD[:]
    _build.build_hip(jobs=2)
    assert _build.LAST_BUILD == []
    # a touch alone (content unchanged, older mtime) is not an edit
    subprocess.run(["touch", "-d", "2000-01-01", str(src)], check=True)
    _build.build_hip(jobs=2)
    assert _build.LAST_BUILD == []
    # an edit whose file is OLDER than the objects (a snapshot's checkout order) still recompiles
    src.write_text(KERNEL % "2.0f")
    subprocess.run(["touch", "-d", "2000-01-01", str(src)], check=True)
    _build.build_hip(jobs=2)
    assert _build.LAST_BUILD == ["csrc/build/probe.hip.o", "libk8srca_hip.so"]
    # a header edit rebuilds every kernel object
    del _build.LAST_BUILD[:]
    (pkg / "csrc" / "kernels" / "probe.h").write_text("// header v2\n")
    subprocess.run(["touch", "-d", "2000-01-01", str(pkg / "csrc" / "kernels" / "probe.h")], check=True)
    _build.build_hip(jobs=2)
    assert "csrc/build/probe.hip.o" in _build.LAST_BUILD


def test_driver_build_forces_a_full_compile(monkeypatch):
    import __graft_entry__ as g
    calls = []
    monkeypatch.setattr(_build, "build_all", lambda force=False: calls.append(force) or ["x.so"])
    g.build()
    assert calls == [True]


def test_arch_and_compiler_come_from_knobs():
    from k8s_llm_rca_amd.knobs import KNOBS
    assert _build.ARCH == KNOBS.offload_arch == "gfx950"
    assert _build.HIPCC == KNOBS.hipcc
    text = open(_build.__file__).read()
    assert "os.environ" not in text

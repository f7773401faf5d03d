"""knobs.py: one typed place for every runtime switch (VERDICT r4 hygiene)."""
import os
import re
import subprocess
import sys

import pytest
import torch

from k8s_llm_rca_amd import knobs as K

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "k8s_llm_rca_amd")


def test_from_env_parses_types_and_legacy_names():
    k = K.Knobs.from_env({"K8SRCA_PF_W8": "5", "K8SRCA_SKINNY": "0", "K8SRCA_PF_OVERHEAD_PAGES": "3.5",
                          "K8S_RCA_AR_MAX_MB": "16", "K8SRCA_SHAPE_TRACE": "/tmp/x.jsonl"})
    assert k.pf_w8 == 5 and k.skinny is False and k.pf_overhead_pages == 3.5
    assert k.ar_max_mb == 16                      # legacy name honoured
    assert k.shape_trace == "/tmp/x.jsonl"
    assert k.describe()["K8SRCA_PF_W8"] == 5
    # the new name wins over the legacy one
    assert K.Knobs.from_env({"K8S_RCA_AR_MAX_MB": "16", "K8SRCA_AR_MAX_MB": "32"}).ar_max_mb == 32


def test_override_restores():
    before = (K.KNOBS.pf_w8, K.KNOBS.glds_hand)
    with K.override(pf_w8=2, glds_hand=False):
        assert (K.KNOBS.pf_w8, K.KNOBS.glds_hand) == (2, False)
    assert (K.KNOBS.pf_w8, K.KNOBS.glds_hand) == before
    with pytest.raises(AttributeError):
        with K.override(no_such_knob=1):
            pass


def test_native_knobs_reach_the_library():
    from k8s_llm_rca_amd.ops import _lib
    if not _lib.available():
        pytest.skip("HIP library not built")
    L = _lib.lib()
    slot = K.NATIVE["pf_w8"]
    with K.override(pf_w8=4):
        assert L.k8s_get_knob(slot) == 4
    assert L.k8s_get_knob(slot) == K.KNOBS.pf_w8


def test_environment_read_in_one_place():
    """No module under ops/, engine/, models/, parallel/ or csrc/ reads an
    environment variable of ours: knobs.py does (placement's *_VISIBLE_DEVICES
    and torchrun's RANK / WORLD_SIZE contract are not ours)."""
    offenders = []
    pat = re.compile(r"(os\.environ|getenv)\s*[\.\[(]\s*(get\()?\s*\"(K8S[A-Z_]*)")
    for sub in ("ops", "engine", "models", "parallel", "csrc/kernels", "graph", "utils", "bench"):
        d = os.path.join(PKG, sub)
        for f in os.listdir(d):
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                for i, line in enumerate(open(os.path.join(d, f)), 1):
                    if pat.search(line):
                        offenders.append(f"{sub}/{f}:{i}")
    assert not offenders, offenders


def test_env_applies_in_a_fresh_process():
    code = "from k8s_llm_rca_amd.knobs import KNOBS; print(KNOBS.pf_target_wgs, KNOBS.step_timing)"
    env = dict(os.environ, K8SRCA_PF_TARGET_WGS="256", K8SRCA_STEP_TIMING="1")
    out = subprocess.check_output([sys.executable, "-c", code], env=env, cwd=ROOT, text=True).split()
    assert out == ["256", "True"]


def test_nonfinite_flag_cpu_reference():
    from k8s_llm_rca_amd.ops.norm import nonfinite_flag
    f = torch.zeros(1, dtype=torch.int32)
    nonfinite_flag(torch.ones(4, 8), f)
    assert int(f[0]) == 0
    x = torch.ones(4, 8)
    x[2, 3] = float("inf")
    nonfinite_flag(x, f)
    assert int(f[0]) == 1


def test_poison_scratch_fills_nan():
    from k8s_llm_rca_amd.ops._lib import scratch
    with K.override(poison=True):
        t = scratch(16, torch.float32, "cpu")
        assert torch.isnan(t).all()
        assert scratch(4, torch.int32, "cpu").dtype == torch.int32  # integer buffers are not poisoned
    assert scratch((2, 3), torch.bfloat16, "cpu").shape == (2, 3)


def test_import_time_knobs_refuse_runtime_changes():
    """knobs copied into a module constant at import (layer_exec._norm_fuse,
    linear.SKINNY_MAX_M, ...) would change KNOBS with no effect: override / set_knob
    refuse them and name the constant."""
    assert "norm_fuse" in K.AT_IMPORT and "skinny_max_m" in K.AT_IMPORT
    with pytest.raises(ValueError, match="layer_exec._norm_fuse"):
        with K.override(norm_fuse=False):
            pass
    with pytest.raises(ValueError, match="SKINNY_MAX_M"):
        K.set_knob("skinny_max_m", "8")
    assert K.KNOBS.norm_fuse is True and K.KNOBS.skinny_max_m == 16
    # every at-import knob really is copied at import: its name appears in the module it names
    for name, where in K.AT_IMPORT.items():
        parts = where.split(" ")[0].split(".")
        paths = [os.path.join(PKG, *parts[:i]) + ".py" for i in range(len(parts), 0, -1)]
        path = next(p for p in paths if os.path.exists(p))
        assert f"KNOBS.{name}" in open(path).read(), (name, path)

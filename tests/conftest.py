import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# prompt prefill batching holds prompts back by WALL-CLOCK time, so which step
# a prompt lands in would vary run to run; tests that compare two engines'
# tokens need identical step composition.  The batching itself has its own
# tests (test_engine.py::test_prompt_prefill_batching_defers_then_runs).
os.environ.setdefault("K8SRCA_PREFILL_MIN", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: longer CPU tests")


@pytest.fixture
def knob():
    """``knob(name, value)``: set a k8s_llm_rca_amd.knobs switch for this test
    (native ones pushed to the HIP library); restored at teardown."""
    from k8s_llm_rca_amd import knobs as K
    old = {}

    def set_(name, value):
        K._runtime_settable(name)  # a knob copied into a module constant at import cannot be set here
        if name not in old:
            old[name] = getattr(K.KNOBS, name)
        setattr(K.KNOBS, name, value)
        if name in K.NATIVE:
            K.push_native()

    yield set_
    for name, v in old.items():
        setattr(K.KNOBS, name, v)
    if any(n in K.NATIVE for n in old):
        K.push_native()


@pytest.fixture(scope="session")
def small_cluster():
    from k8s_llm_rca_amd.graph.synth import generate_cluster
    return generate_cluster(3000, 20, seed=2)

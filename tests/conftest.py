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


@pytest.fixture(scope="session")
def small_cluster():
    from k8s_llm_rca_amd.graph.synth import generate_cluster
    return generate_cluster(3000, 20, seed=2)

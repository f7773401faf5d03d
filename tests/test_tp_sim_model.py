"""The xGMI cost model behind ``bench --tp-sim`` (parallel/tpsim.py): hop
latency enters once per fabric hand-off, so the sensitivity the projection
reports (2.5 / 5 / 10 us) scales as the model says."""
import pytest

from k8s_llm_rca_amd.parallel import tpsim as T


def test_hop_latency_terms():
    nb, n = 2 << 20, 8
    for mode, hops in ((1, 1), (2, 2), (0, 2 * (n - 1))):
        a, b = T.xgmi_model_us(nb, n, mode, 2.5), T.xgmi_model_us(nb, n, mode, 10.0)
        assert b - a == pytest.approx(7.5 * hops)
    assert T.xgmi_model_us(nb, n, 2) == T.xgmi_model_us(nb, n, 2, T.XGMI_HOP_US)
    assert T.a2a_model_us(nb, n, 10.0) - T.a2a_model_us(nb, n, 2.5) == pytest.approx(7.5)
    # bandwidth terms: one-shot moves the whole message over one link, two-shot 2/N of it
    assert T.xgmi_model_us(nb, n, 1, 0.0) == pytest.approx(nb / (T.XGMI_LINK_GBPS * 1e3))
    assert T.xgmi_model_us(nb, n, 2, 0.0) == pytest.approx(2 * nb / (n * T.XGMI_LINK_GBPS * 1e3))
    assert tuple(T.HOP_SENSITIVITY_US) == (2.5, 5.0, 10.0)


def test_fused_standin_selection_follows_the_executor():
    """The projection times the fused all-reduce + add + RMSNorm exactly where the
    layer executor would fuse (message + row sums fit the buffer; two-shot needs
    H / 8 chunks divisible by the world), else the plain all-reduce."""
    class Car:
        max_bytes, world = 8 << 20, 8

        def addnorm(self, *a, **k):  # presence is what the selection checks
            return None
    car, H = Car(), 8192
    assert T._fused_epilogue(car, 32, H, 1) and T._fused_epilogue(car, 256, H, 2)
    assert not T._fused_epilogue(car, 512, H, 2)      # 8 MiB + row sums > the buffer
    assert not T._fused_epilogue(car, 32, H, 0)       # RCCL-size message
    assert not T._fused_epilogue(car, 32, 8200, 2)    # 1025 chunks do not split over 8 ranks
    assert not T._fused_epilogue(None, 32, H, 1)

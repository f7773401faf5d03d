"""Sampling semantics (B9/B10) on the fp32 reference path: top-k / top-p
restrictions, their empirical distribution, and the vocab-parallel candidate
combine against the single-device result."""
import math

import pytest
import torch

from k8s_llm_rca_amd.ops import sampling as SMP


def _args(B, temps, k, p, seeds=None, steps=None):
    return dict(temperature=torch.tensor(temps, dtype=torch.float32),
                seeds=torch.arange(B, dtype=torch.int32) * 7 + 1 if seeds is None else seeds,
                steps=torch.zeros(B, dtype=torch.int32) if steps is None else steps,
                mask_id=torch.full((B,), -1, dtype=torch.int32), mask_table=None,
                list_off=torch.zeros(B, dtype=torch.int32), list_len=torch.zeros(B, dtype=torch.int32),
                lists=torch.zeros(1, dtype=torch.int32),
                top_k=torch.tensor(k, dtype=torch.int32), top_p=torch.tensor(p, dtype=torch.float32))


def _naive_nucleus(v, p):
    """HF-style top-p keep mask: sort desc, keep the prefix whose mass before the token is < p."""
    pr = torch.softmax(v.double(), 0)
    order = torch.argsort(v, descending=True)
    before = torch.cumsum(pr[order], 0) - pr[order]
    keep = torch.zeros_like(v, dtype=torch.bool)
    keep[order[before < p]] = True
    return keep


def test_filter_threshold_matches_naive():
    g = torch.Generator().manual_seed(0)
    for trial in range(20):
        v = torch.randn(3000, generator=g) * (0.5 + trial / 5)
        for k in (1, 5, 64, 0):
            for p in (0.3, 0.9, 1.0):
                keep = SMP.filter_threshold(v, k, p)
                ref = torch.ones_like(keep)
                if k:
                    ref &= v >= torch.topk(v, k).values[-1]
                if p < 1:
                    sub = torch.where(ref, v, torch.full_like(v, -float("inf")))
                    ref &= _naive_nucleus(sub, p)
                assert torch.equal(keep, ref), (trial, k, p)


def test_topk_topp_restrict_and_distribution():
    V, n = 512, 4000
    torch.manual_seed(1)
    base = torch.randn(V) * 2
    logits = base.repeat(n, 1)
    temps = [0.8] * n
    a = _args(n, temps, [8] * n, [0.9] * n, seeds=torch.arange(n, dtype=torch.int32) * 13 + 5)
    out = torch.empty(n, dtype=torch.int32)
    SMP._sample_ref(logits, a["temperature"], a["seeds"], a["steps"], a["mask_id"], None, a["list_off"],
                    a["list_len"], a["lists"], V, out, top_k=a["top_k"], top_p=a["top_p"])
    v = base / 0.8
    keep = SMP.filter_threshold(v, 8, 0.9)
    assert bool(keep[out.long()].all())
    probs = torch.where(keep, torch.softmax(v.double(), 0), torch.zeros(V, dtype=torch.float64))
    probs /= probs.sum()
    counts = torch.bincount(out.long(), minlength=V).double()
    expect = probs * n
    idx = expect > 0
    chi2 = float((((counts[idx] - expect[idx]) ** 2) / expect[idx]).sum())
    dof = int(idx.sum()) - 1
    assert chi2 < dof + 6 * math.sqrt(2 * dof) + 10, (chi2, dof)


@pytest.mark.parametrize("tp", [2, 4])
def test_candidates_combine_matches_single_device(tp):
    B, V = 6, 4096
    torch.manual_seed(2)
    logits = torch.randn(B, V)
    logits[[1, 3, 4]] *= 8  # peaked rows: their nuclei hold < CAND_K tokens per shard
    temps = [0.7, 1.0, 0.5, 1.2, 0.9, 0.0]
    ks = [5, 64, 1, 20, 0, 10]
    ps = [1.0, 0.95, 1.0, 0.5, 0.3, 1.0]
    a = _args(B, temps, ks, ps, steps=torch.arange(B, dtype=torch.int32) + 3)
    full = torch.empty(B, dtype=torch.int32)
    SMP._sample_ref(logits, a["temperature"], a["seeds"], a["steps"], a["mask_id"], None, a["list_off"],
                    a["list_len"], a["lists"], V, full, top_k=a["top_k"], top_p=a["top_p"])
    vl = V // tp
    pairs, cands = [], []
    for r in range(tp):
        o, c = SMP.sample(logits[:, r * vl:(r + 1) * vl].contiguous(), a["temperature"], a["seeds"], a["steps"],
                          a["mask_id"], None, a["list_off"], a["list_len"], a["lists"], V, vocab_off=r * vl,
                          pairs=True, top_k=a["top_k"], top_p=a["top_p"], candidates=True)
        pairs.append(o)
        cands.append(c)
    tok = SMP.combine_pairs(torch.stack(pairs))
    filt = (a["top_k"] > 0) | (a["top_p"] < 1)
    ct = SMP.combine_candidates(torch.stack(cands), a["top_k"], a["top_p"])
    got = torch.where(filt, ct, tok)
    assert torch.equal(got, full), (got, full)


def _nonfinite_case(dev):
    B, V = 5, 1024
    torch.manual_seed(4)
    logits = torch.randn(B, V)
    logits[0, 17] = float("nan")     # allowed NaN -> NON_FINITE
    logits[1, 900] = float("inf")    # allowed +inf -> NON_FINITE
    logits[2, 3] = -float("inf")     # allowed -inf -> NON_FINITE (the model's output went bad)
    logits[3, 40] = float("nan")     # NaN only in a token the row's list excludes -> a normal pick
    lists = torch.tensor([1, 2, 3, 5, 8], dtype=torch.int32)
    a = _args(B, [0.0, 0.7, 0.0, 0.9, 0.0], [0] * B, [1.0] * B)
    a["list_len"][3] = len(lists)
    a["lists"] = lists
    out = torch.empty(B, dtype=torch.int32, device=dev)
    return logits.to(dev), a, out, V


def test_sampler_flags_nonfinite_rows_reference():
    """A row whose allowed logits are not all finite returns SMP.NON_FINITE (the
    engine then fails that request: engine._process_tokens) instead of a token
    picked from garbage; NaN outside the allowed set does not matter."""
    logits, a, out, V = _nonfinite_case("cpu")
    SMP._sample_ref(logits, a["temperature"], a["seeds"], a["steps"], a["mask_id"], None, a["list_off"],
                    a["list_len"], a["lists"], V, out)
    assert out[:3].tolist() == [SMP.NON_FINITE] * 3
    assert int(out[3]) in (1, 2, 3, 5, 8) and 0 <= int(out[4]) < V
    pairs = torch.empty(5, 2)
    SMP._sample_ref(logits, a["temperature"], a["seeds"], a["steps"], a["mask_id"], None, a["list_off"],
                    a["list_len"], a["lists"], V, pairs, pairs=True)
    # a bad shard's +inf wins the cross-shard max: the TP combine returns NON_FINITE too
    assert SMP.combine_pairs(torch.stack([pairs, pairs])).tolist()[:3] == [SMP.NON_FINITE] * 3


@pytest.mark.parametrize("tp", [2, 4])
def test_tp_candidates_keep_nonfinite_flag(tp):
    """under TP a top-k row whose logits are NaN in ONE
    shard must come out of the combine as NON_FINITE -- the candidates path
    must not replace the flag with a token picked from the poisoned logits."""
    B, V = 4, 2048
    torch.manual_seed(9)
    logits = torch.randn(B, V)
    vl = V // tp
    logits[1, vl + 5] = float("nan")   # row 1: NaN in shard 1 only, a top-k row
    logits[2, 7] = float("inf")        # row 2: +inf in shard 0, a top-k row
    a = _args(B, [0.8, 0.8, 0.8, 0.8], [8, 8, 16, 0], [1.0, 0.9, 1.0, 1.0])
    pairs, cands = [], []
    for r in range(tp):
        o, c = SMP.sample(logits[:, r * vl:(r + 1) * vl].contiguous(), a["temperature"], a["seeds"], a["steps"],
                          a["mask_id"], None, a["list_off"], a["list_len"], a["lists"], V, vocab_off=r * vl,
                          pairs=True, top_k=a["top_k"], top_p=a["top_p"], candidates=True)
        pairs.append(o)
        cands.append(c)
    sel = (a["top_k"] > 0) & (a["top_k"] <= SMP.CAND_K)
    got = SMP.combine_shards(torch.stack(pairs), torch.stack(cands), sel, a["top_k"], a["top_p"])
    assert got[1].item() == SMP.NON_FINITE and got[2].item() == SMP.NON_FINITE
    assert got[0].item() >= 0 and got[3].item() >= 0
    # the healthy rows equal the single-device pick
    full = torch.empty(B, dtype=torch.int32)
    SMP._sample_ref(logits, a["temperature"], a["seeds"], a["steps"], a["mask_id"], None, a["list_off"],
                    a["list_len"], a["lists"], V, full, top_k=a["top_k"], top_p=a["top_p"])
    assert got[0] == full[0] and got[3] == full[3]


@pytest.mark.gpu
def test_sampler_flags_nonfinite_rows_kernel():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    logits, a, out, V = _nonfinite_case("cuda")
    a = {k: (v.cuda() if isinstance(v, torch.Tensor) else v) for k, v in a.items()}
    for lg in (logits, logits.bfloat16()):
        ref = torch.empty(5, dtype=torch.int32)
        SMP._sample_ref(lg.float().cpu(), *(a[k].cpu() for k in ("temperature", "seeds", "steps", "mask_id")), None,
                        a["list_off"].cpu(), a["list_len"].cpu(), a["lists"].cpu(), V, ref)
        got = SMP.sample(lg, a["temperature"], a["seeds"], a["steps"], a["mask_id"], None, a["list_off"],
                         a["list_len"], a["lists"], V)
        assert got.cpu().tolist()[:3] == [SMP.NON_FINITE] * 3
        assert torch.equal(got.cpu()[3:], ref[3:])


def test_mask_mirror_never_skips_a_row_registered_during_upload():
    """The device mirror of the grammar bitmaps (SamplerMixin._mask_table) used
    to read the table's rows and THEN its version: a row registered by another
    thread in between was counted as uploaded, so the mirror was never
    refreshed for it and sampling read past the table (garbage bits: runs that
    end at once with no error).  Rows and version are now taken together."""
    import numpy as np
    import torch
    from k8s_llm_rca_amd.engine.sampler import SamplerMixin
    from k8s_llm_rca_amd.engine.structured import MaskTable

    mt = MaskTable(64)
    mt.get(("a",), lambda: np.ones(64, bool))

    class Racy(MaskTable):
        fired = False

        def snapshot(self):
            out = super().snapshot()
            if not Racy.fired:  # another thread registers a mask right after the rows were stacked
                Racy.fired = True
                self.get(("b",), lambda: np.zeros(64, bool))
            return out

    racy = Racy(64)
    racy.get(("a",), lambda: np.ones(64, bool))

    class G:
        masks = racy

    class Eng(SamplerMixin):
        def __init__(self):
            self.grt, self.device, self._mask_ver, self._mask_dev = G(), torch.device("cpu"), -1, None

    e = Eng()
    t1 = e._mask_table()
    assert t1.shape[0] == 1 and racy.version == 2
    t2 = e._mask_table()  # the version it recorded is the rows', so the new row is picked up now
    assert t2.shape[0] == 2

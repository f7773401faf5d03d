"""Masked greedy / temperature / top-k / top-p sampling (B9) with grammar masks.

The HIP kernel (``csrc/kernels/sampling.hip``) reads fp32 (default) or bf16
logits; ``_sample_ref`` is its fp32 PyTorch mirror (same noise, same order
key, same threshold rules) used on CPU tensors and by the tests.
"""
from __future__ import annotations

from typing import Optional

import torch

from ._lib import check, lib, ptr, stream_ptr, use_hip

CAND_K = 64  # per-rank candidates of a vocab-parallel top-k / top-p row (k <= 64)


def sample(logits: torch.Tensor, temperature: Optional[torch.Tensor], seeds: Optional[torch.Tensor],
           steps: Optional[torch.Tensor], mask_id: Optional[torch.Tensor], mask_table: Optional[torch.Tensor],
           list_off: Optional[torch.Tensor], list_len: Optional[torch.Tensor], lists: Optional[torch.Tensor],
           vocab: int, out: Optional[torch.Tensor] = None, vocab_off: int = 0,
           pairs: bool = False, top_k: Optional[torch.Tensor] = None, top_p: Optional[torch.Tensor] = None,
           candidates: bool = False):
    """One token per row of ``logits`` [B, ld] (fp32 or bf16).

    Row b is restricted to ``lists[list_off[b]:list_off[b]+list_len[b]]`` when
    ``list_len[b] > 0``, else to the allow-bitmap ``mask_table[mask_id[b]]``
    (``mask_id[b] < 0``: unrestricted), then to its top-``top_k[b]`` (``<= 0``:
    off) and its top-``top_p[b]`` nucleus (``>= 1``: off).
    ``temperature[b] <= 0`` is greedy (top-k / top-p do not change an argmax).

    Vocab-parallel use: ``logits`` holds global columns ``vocab_off ..``; with
    ``pairs=True`` the result is [B, 2] float32 (winning perturbed score,
    global id; -inf / -1 when the shard has no allowed token; +inf /
    ``NON_FINITE`` when an allowed logit is NaN / inf) to be combined across
    ranks by :func:`combine_pairs`.  A row with a non-finite allowed logit
    samples ``NON_FINITE`` (-2): the engine fails its request.  ``candidates=True`` (with pairs)
    also returns [B, CAND_K, 3] (v, id, v + Gumbel noise) shard candidates of
    the top-k / top-p rows for :func:`combine_candidates`.
    """
    B = logits.shape[0]
    V = max(0, min(logits.shape[1], vocab - vocab_off))
    if pairs:
        out = torch.empty(B, 2, dtype=torch.float32, device=logits.device)
    elif out is None:
        out = torch.empty(B, dtype=torch.int32, device=logits.device)
    cand = torch.empty(B, CAND_K, 3, dtype=torch.float32, device=logits.device) if candidates else None
    if use_hip(logits):
        assert logits.dtype in (torch.bfloat16, torch.float32) and logits.stride(1) == 1 and vocab_off % 8 == 0
        assert top_k is None or top_k.dtype == torch.int32
        assert top_p is None or top_p.dtype == torch.float32
        words = mask_table.shape[1] if mask_table is not None else 0
        if mask_table is not None:
            assert mask_table.dtype == torch.int32 and words * 32 >= vocab
        check(lib().k8s_sample(ptr(logits), logits.stride(0), B, V, vocab_off, ptr(temperature), ptr(seeds),
                               ptr(steps), ptr(mask_id), ptr(mask_table), words, ptr(list_off), ptr(list_len),
                               ptr(lists), 0 if pairs else ptr(out), ptr(out) if pairs else 0,
                               stream_ptr(logits), int(logits.dtype == torch.float32), ptr(top_k), ptr(top_p),
                               ptr(cand), CAND_K if candidates else 0), "sample")
        return (out, cand) if candidates else out
    _sample_ref(logits, temperature, seeds, steps, mask_id, mask_table, list_off, list_len, lists, V, out,
                vocab_off, pairs, top_k, top_p, cand)
    return (out, cand) if candidates else out


def combine_pairs(gathered: torch.Tensor) -> torch.Tensor:
    """[tp, B, 2] per-rank (score, id) winners -> [B] int32 token ids.  Ranks
    hold increasing vocab ranges, so the first maximum is also the smallest id
    (the single-device kernel's tie rule)."""
    best = gathered[:, :, 0].argmax(dim=0)
    ids = gathered[:, :, 1].gather(0, best[None, :])[0]
    return ids.round().to(torch.int32)


def combine_candidates(cands: torch.Tensor, top_k: torch.Tensor, top_p: torch.Tensor) -> torch.Tensor:
    """[tp, B, C, 3] per-rank (v, id, v + G) candidates of top-k / top-p rows ->
    [B] int32 tokens: the same top-k / nucleus rules as the kernel over the
    union of the ranks' candidates, then the max of the kernel's own perturbed
    scores (identical on every rank).  Exact for rows with ``0 < top_k <=
    CAND_K``: the whole top-k set, hence the nucleus and its mass, is in the
    union.  The engine sends every other filtered row through a logits
    all-gather instead (``VocabParallelSampler._sample_gathered``, engine/tp_sampler.py)."""
    tp, B, C, _ = cands.shape
    allc = cands.permute(1, 0, 2, 3).reshape(B, tp * C, 3)
    v, ids, sc = allc[..., 0], allc[..., 1].round().long(), allc[..., 2]
    valid = ids >= 0
    v = torch.where(valid, v, torch.full_like(v, -float("inf")))
    # order: v desc, id asc
    key = torch.where(valid, ids, torch.full_like(ids, 1 << 30))
    order = torch.argsort(key, dim=1, stable=True)
    v, ids, valid, sc = v.gather(1, order), ids.gather(1, order), valid.gather(1, order), sc.gather(1, order)
    order = torch.argsort(v, dim=1, descending=True, stable=True)
    v, ids, valid, sc = v.gather(1, order), ids.gather(1, order), valid.gather(1, order), sc.gather(1, order)
    keep = valid.clone()
    k = top_k.long().clamp(min=0)
    n = keep.sum(1)
    kth = torch.where((k > 0) & (k < n), v.gather(1, (k - 1).clamp(min=0).view(-1, 1)).view(-1),
                      torch.full_like(v[:, 0], -float("inf")))
    keep &= v >= kth[:, None]
    vmax = v[:, 0:1]
    w = torch.where(keep, torch.exp(v - vmax), torch.zeros_like(v))
    z = w.sum(1, keepdim=True)
    before = torch.cumsum(w, 1) - w  # mass strictly above (sorted order)
    p = top_p.float().view(-1, 1)
    keep &= (p >= 1.0) | (before < p * z)
    # ties with the last kept value stay (threshold rule)
    last = torch.where(keep, v, torch.full_like(v, float("inf"))).min(1, keepdim=True).values
    keep = valid & (v >= last) & (v >= kth[:, None])
    score = torch.where(keep, sc, torch.full_like(sc, -float("inf")))
    best = score.max(1, keepdim=True).values
    first = torch.where(score == best, ids, torch.full_like(ids, 1 << 30)).min(1).values
    return first.to(torch.int32)


def combine_shards(pairs: torch.Tensor, cands: Optional[torch.Tensor], cand_rows: Optional[torch.Tensor],
                   top_k: Optional[torch.Tensor], top_p: Optional[torch.Tensor]) -> torch.Tensor:
    """The TP sampler's combine (``VocabParallelSampler._sample_shard``): [tp, B, 2]
    winners -> [B] tokens, and for the ``cand_rows`` (bool [B]: top-k rows with
    ``k <= CAND_K``) the exact top-k / top-p pick from the [tp, B, C, 3]
    candidates.  A row that any shard flagged ``NON_FINITE`` keeps the flag:
    its candidates come from the same poisoned logits (NaN fails every
    comparison), so they would hand back a token picked from garbage."""
    tok = combine_pairs(pairs)
    if cands is None:
        return tok
    ct = combine_candidates(cands, top_k, top_p)
    return torch.where(cand_rows & (tok != NON_FINITE), ct, tok)


def _mix32(x: torch.Tensor) -> torch.Tensor:
    M = 0xFFFFFFFF
    x = x & M
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & M
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & M
    x = x ^ (x >> 16)
    return x


def gumbel_ref(seed: int, row: int, step: int, idx: torch.Tensor) -> torch.Tensor:
    """Bit-exact host mirror of the kernel's noise (int64 arithmetic)."""
    M = 0xFFFFFFFF
    i = _mix32(idx.long() + 0x27D4EB2F)
    s = _mix32(torch.tensor((step * 0x85EBCA6B) & M) ^ i)
    r = _mix32(torch.tensor((row * 0x9E3779B9) & M) ^ s)
    h = _mix32(torch.tensor(seed & M) ^ r)
    u = ((h >> 8).double() + 0.5) * (1.0 / 16777216.0)
    return (-torch.log(-torch.log(u.float()))).float()


def _okey(v: torch.Tensor) -> torch.Tensor:
    """The kernel's order-preserving uint32 image of float32 ``v`` (as int64)."""
    u = v.float().contiguous().view(torch.int32).long() & 0xFFFFFFFF
    return torch.where(u >= 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)


def filter_threshold(v: torch.Tensor, k: int, p: float) -> torch.Tensor:
    """Boolean keep-mask of allowed values ``v`` (fp32, temperature-scaled) under
    top-``k`` then top-``p``: keys >= the k-th largest key, then the smallest
    highest-key prefix whose softmax mass reaches ``p`` (ties kept)."""
    key = _okey(v)
    keep = torch.ones_like(key, dtype=torch.bool)
    if 0 < k < v.numel():
        kth = torch.sort(key, descending=True).values[k - 1]
        keep &= key >= kth
    if p < 1.0 and keep.any():
        vv = v[keep].double()
        kk = key[keep]
        w = torch.exp(vv - vv.max())
        order = torch.argsort(kk, descending=True, stable=True)
        ks, ws = kk[order], w[order]
        target = p * ws.sum()
        cum = torch.cumsum(ws, 0)
        j = int(torch.nonzero(cum >= target).flatten()[0]) if bool((cum >= target).any()) else len(ws) - 1
        keep &= key >= ks[j]
    return keep


# token id a sampler returns for a row whose allowed logits are not all finite
# (csrc/kernels/sampling.hip kNonFinite); -1 = no allowed token
NON_FINITE = -2


def _sample_ref(logits, temperature, seeds, steps, mask_id, mask_table, list_off, list_len, lists, vocab, out,
                vocab_off=0, pairs=False, top_k=None, top_p=None, cand=None):
    """``vocab`` = local columns to consider; ids are global (``+ vocab_off``)."""
    B = logits.shape[0]
    for b in range(B):
        lg = logits[b, :vocab].float()
        temp = float(temperature[b]) if temperature is not None else 0.0
        ll = int(list_len[b]) if list_len is not None else 0
        if ll > 0:
            o = int(list_off[b])
            c = lists[o:o + ll].long() - vocab_off
            c = c[(c >= 0) & (c < vocab)]
        else:
            mid = int(mask_id[b]) if mask_id is not None else -1
            if mid >= 0:
                words = mask_table[mid].long() & 0xFFFFFFFF
                bits = ((words[:, None] >> torch.arange(32)[None, :]) & 1).reshape(-1)
                c = torch.nonzero(bits[vocab_off:vocab_off + vocab].bool()).flatten()
            else:
                c = torch.arange(vocab)
        k = int(top_k[b]) if top_k is not None else 0
        p = float(top_p[b]) if top_p is not None else 1.0
        it = torch.tensor(1.0, dtype=torch.float32) if temp <= 0 else (1.0 / torch.tensor(temp, dtype=torch.float32))
        v = lg[c] * it
        if cand is not None:
            cand[b, :, 0] = -float("inf")
            cand[b, :, 1] = -1.0
            cand[b, :, 2] = -float("inf")
            if (k > 0 or p < 1.0) and len(c):
                keff = k if 0 < k < cand.shape[1] else cand.shape[1]
                keep = filter_threshold(v, keff, 1.0)
                cv, ci = v[keep], c[keep] + vocab_off
                order = torch.argsort(ci, stable=True)
                cv, ci = cv[order], ci[order]
                order = torch.argsort(cv, descending=True, stable=True)
                cv, ci = cv[order][:cand.shape[1]], ci[order][:cand.shape[1]]
                cand[b, :len(cv), 0] = cv
                cand[b, :len(cv), 1] = ci.float()
                cand[b, :len(cv), 2] = cv + gumbel_ref(int(seeds[b]), 0, int(steps[b]), ci) if temp > 0 else cv
        if len(c) and not bool(torch.isfinite(v).all()):  # the kernel's kNonFinite row
            if pairs:
                out[b, 0], out[b, 1] = float("inf"), float(NON_FINITE)
            else:
                out[b] = NON_FINITE
            continue
        if len(c) and temp > 0 and (k > 0 or p < 1.0):
            keep = filter_threshold(v, k, p)
            c, v = c[keep], v[keep]
        if len(c) == 0:
            if pairs:
                out[b, 0], out[b, 1] = -float("inf"), -1.0
            else:
                out[b] = -1
            continue
        if temp > 0:
            v = v + gumbel_ref(int(seeds[b]), 0, int(steps[b]), c + vocab_off)
        best = torch.max(v)
        tok = int(c[torch.nonzero(v == best).flatten()[0]]) + vocab_off
        if pairs:
            out[b, 0], out[b, 1] = float(best), float(tok)
        else:
            out[b] = tok
    return out

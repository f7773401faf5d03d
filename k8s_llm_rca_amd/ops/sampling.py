"""Masked greedy / Gumbel-max sampling (B9) with grammar masks."""
from __future__ import annotations

from typing import Optional

import torch

from ._lib import check, lib, ptr, stream_ptr, use_hip


def sample(logits: torch.Tensor, temperature: Optional[torch.Tensor], seeds: Optional[torch.Tensor],
           steps: Optional[torch.Tensor], mask_id: Optional[torch.Tensor], mask_table: Optional[torch.Tensor],
           list_off: Optional[torch.Tensor], list_len: Optional[torch.Tensor], lists: Optional[torch.Tensor],
           vocab: int, out: Optional[torch.Tensor] = None, vocab_off: int = 0,
           pairs: bool = False) -> torch.Tensor:
    """One token per row of ``logits`` [B, ld] (bf16).

    Row b is restricted to ``lists[list_off[b]:list_off[b]+list_len[b]]`` when
    ``list_len[b] > 0``, else to the allow-bitmap ``mask_table[mask_id[b]]``
    (``mask_id[b] < 0``: unrestricted).  ``temperature[b] <= 0`` is greedy.

    Vocab-parallel use: ``logits`` holds global columns ``vocab_off ..``; with
    ``pairs=True`` the result is [B, 2] float32 (winning perturbed score,
    global id; -inf / -1 when the shard has no allowed token) to be combined
    across ranks by :func:`combine_pairs`.
    """
    B = logits.shape[0]
    V = max(0, min(logits.shape[1], vocab - vocab_off))
    if pairs:
        out = torch.empty(B, 2, dtype=torch.float32, device=logits.device)
    elif out is None:
        out = torch.empty(B, dtype=torch.int32, device=logits.device)
    if use_hip(logits):
        assert logits.dtype == torch.bfloat16 and logits.stride(1) == 1 and vocab_off % 8 == 0
        words = mask_table.shape[1] if mask_table is not None else 0
        if mask_table is not None:
            assert mask_table.dtype == torch.int32 and words * 32 >= vocab
        check(lib().k8s_sample(ptr(logits), logits.stride(0), B, V, vocab_off, ptr(temperature), ptr(seeds),
                               ptr(steps), ptr(mask_id), ptr(mask_table), words, ptr(list_off), ptr(list_len),
                               ptr(lists), 0 if pairs else ptr(out), ptr(out) if pairs else 0,
                               stream_ptr(logits)), "sample")
        return out
    return _sample_ref(logits, temperature, seeds, steps, mask_id, mask_table, list_off, list_len, lists, V, out,
                       vocab_off, pairs)


def combine_pairs(gathered: torch.Tensor) -> torch.Tensor:
    """[tp, B, 2] per-rank (score, id) winners -> [B] int32 token ids.  Ranks
    hold increasing vocab ranges, so the first maximum is also the smallest id
    (the single-device kernel's tie rule)."""
    best = gathered[:, :, 0].argmax(dim=0)
    ids = gathered[:, :, 1].gather(0, best[None, :])[0]
    return ids.round().to(torch.int32)


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


def _sample_ref(logits, temperature, seeds, steps, mask_id, mask_table, list_off, list_len, lists, vocab, out,
                vocab_off=0, pairs=False):
    """``vocab`` = local columns to consider; ids are global (``+ vocab_off``)."""
    B = logits.shape[0]
    for b in range(B):
        lg = logits[b, :vocab].float()
        temp = float(temperature[b]) if temperature is not None else 0.0
        ll = int(list_len[b]) if list_len is not None else 0
        if ll > 0:
            o = int(list_off[b])
            cand = lists[o:o + ll].long() - vocab_off
            cand = cand[(cand >= 0) & (cand < vocab)]
        else:
            mid = int(mask_id[b]) if mask_id is not None else -1
            if mid >= 0:
                words = mask_table[mid].long() & 0xFFFFFFFF
                bits = ((words[:, None] >> torch.arange(32)[None, :]) & 1).reshape(-1)
                cand = torch.nonzero(bits[vocab_off:vocab_off + vocab].bool()).flatten()
            else:
                cand = torch.arange(vocab)
        if len(cand) == 0:
            if pairs:
                out[b, 0], out[b, 1] = -float("inf"), -1.0
            else:
                out[b] = -1
            continue
        v = lg[cand]
        if temp > 0:
            v = v / temp + gumbel_ref(int(seeds[b]), 0, int(steps[b]), cand + vocab_off)
        best = torch.max(v)
        tok = int(cand[torch.nonzero(v == best).flatten()[0]]) + vocab_off
        if pairs:
            out[b, 0], out[b, 1] = float(best), float(tok)
        else:
            out[b] = tok
    return out

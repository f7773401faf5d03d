"""Masked greedy / Gumbel-max sampling (B9) with grammar masks."""
from __future__ import annotations

from typing import Optional

import torch

from ._lib import check, lib, ptr, stream_ptr, use_hip


def sample(logits: torch.Tensor, temperature: Optional[torch.Tensor], seeds: Optional[torch.Tensor],
           steps: Optional[torch.Tensor], mask_id: Optional[torch.Tensor], mask_table: Optional[torch.Tensor],
           list_off: Optional[torch.Tensor], list_len: Optional[torch.Tensor], lists: Optional[torch.Tensor],
           vocab: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One token per row of ``logits`` [B, ld] (bf16).

    Row b is restricted to ``lists[list_off[b]:list_off[b]+list_len[b]]`` when
    ``list_len[b] > 0``, else to the allow-bitmap ``mask_table[mask_id[b]]``
    (``mask_id[b] < 0``: unrestricted).  ``temperature[b] <= 0`` is greedy.
    """
    B = logits.shape[0]
    if out is None:
        out = torch.empty(B, dtype=torch.int32, device=logits.device)
    if use_hip(logits):
        assert logits.dtype == torch.bfloat16 and logits.stride(1) == 1
        words = mask_table.shape[1] if mask_table is not None else 0
        if mask_table is not None:
            assert mask_table.dtype == torch.int32 and words * 32 >= vocab
        check(lib().k8s_sample(ptr(logits), logits.stride(0), B, vocab, ptr(temperature), ptr(seeds), ptr(steps),
                               ptr(mask_id), ptr(mask_table), words, ptr(list_off), ptr(list_len), ptr(lists),
                               ptr(out), stream_ptr(logits)), "sample")
        return out
    return _sample_ref(logits, temperature, seeds, steps, mask_id, mask_table, list_off, list_len, lists, vocab, out)


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


def _sample_ref(logits, temperature, seeds, steps, mask_id, mask_table, list_off, list_len, lists, vocab, out):
    B = logits.shape[0]
    for b in range(B):
        lg = logits[b, :vocab].float()
        temp = float(temperature[b]) if temperature is not None else 0.0
        ll = int(list_len[b]) if list_len is not None else 0
        if ll > 0:
            o = int(list_off[b])
            cand = lists[o:o + ll].long()
            cand = cand[(cand >= 0) & (cand < vocab)]
        else:
            mid = int(mask_id[b]) if mask_id is not None else -1
            if mid >= 0:
                words = mask_table[mid].long() & 0xFFFFFFFF
                bits = ((words[:, None] >> torch.arange(32)[None, :]) & 1).reshape(-1)[:vocab].bool()
                cand = torch.nonzero(bits).flatten()
            else:
                cand = torch.arange(vocab)
        if len(cand) == 0:
            out[b] = -1
            continue
        v = lg[cand]
        if temp > 0:
            v = v / temp + gumbel_ref(int(seeds[b]), b, int(steps[b]), cand)
        best = torch.max(v)
        out[b] = int(cand[torch.nonzero(v == best).flatten()[0]])
    return out

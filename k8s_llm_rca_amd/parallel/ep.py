"""Expert parallelism for Mixtral (B15): token dispatch / combine by all-to-all.

Experts are partitioned over the EP group (rank r owns experts
``[r*E/ep, (r+1)*E/ep)``).  Attention runs tensor-parallel, so every rank
holds all T token rows; each rank takes ownership of a contiguous 1/ep of the
rows, and for those:

1. counts exchange -- ``all_to_all_single`` of the per-destination (token, k)
   slot counts (small, fixed size);
2. dispatch -- variable-size ``all_to_all_single`` of the token rows grouped
   by destination rank (+ their local expert ids);
3. grouped SwiGLU on the received rows, sorted by local expert;
4. combine -- the reverse ``all_to_all_single`` returns the expert outputs,
   which are weighted and summed per token (HIP combine kernel on device);
5. ``all_gather`` restores the replicated [T, H] activations.

Over xGMI each all-to-all moves ``T/ep * k * H * 2`` bytes split across the 7
peer links (RCCL), twice per layer.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import moe as M


def ep_moe_forward(moe, li: int, y: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor) -> torch.Tensor:
    pc = moe.pc
    ep, r = pc.ep_size, pc.ep_rank
    grp = pc.ep_group
    T, H = y.shape
    k = moe.k
    per = (T + ep - 1) // ep
    lo, hi = min(T, r * per), min(T, (r + 1) * per)
    n_own = hi - lo
    ids = topk_ids[lo:hi].reshape(-1).long()                       # [n_own*k] global expert ids
    dest = ids // moe.E_local                                        # owning rank of each slot
    order = torch.argsort(dest, stable=True)
    send_counts = torch.bincount(dest, minlength=ep)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=grp)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    tok = (order // k) + lo
    send_x = y.index_select(0, tok)
    send_e = (ids[order] - dest[order] * moe.E_local).to(torch.int32)
    recv_x = y.new_empty((sum(rc), H))
    recv_e = torch.empty(sum(rc), dtype=torch.int32, device=y.device)
    dist.all_to_all_single(recv_x, send_x.contiguous(), rc, sc, group=grp)
    dist.all_to_all_single(recv_e, send_e.contiguous(), rc, sc, group=grp)
    # local grouped experts over the received rows
    out_recv = torch.empty_like(recv_x)
    if recv_x.shape[0]:
        o2, inv2, offs = M.align(recv_e.view(-1, 1), moe.E_local)
        xs = recv_x.index_select(0, o2.long())
        ys = moe.experts(li, xs, offs)
        out_recv = ys.index_select(0, inv2.long())
    back = y.new_empty((sum(sc), H))
    dist.all_to_all_single(back, out_recv.contiguous(), sc, rc, group=grp)
    # un-permute to (token, k) slot order and combine with the routing weights
    y_slots = y.new_empty((n_own * k, H))
    y_slots[order] = back
    inv = torch.arange(n_own * k, dtype=torch.int32, device=y.device)
    own = M.combine(y_slots, inv, topk_w[lo:hi].contiguous(), n_own, k) if n_own else y.new_empty((0, H))
    # restore replicated activations (equal-size all_gather: pad every rank's slice to `per` rows)
    padded = y.new_zeros((per, H))
    padded[:n_own] = own
    parts = [torch.empty_like(padded) for _ in range(ep)]
    dist.all_gather(parts, padded, group=grp)
    return torch.cat(parts, dim=0)[:T]

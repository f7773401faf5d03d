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

Decode-sized batches (``T <= FIXED_MAX_T``), and any batch whose padded
dispatch fits the xGMI communicator's buffer, take :func:`ep_moe_forward_fixed`
instead: fixed-capacity dispatch buffers (every destination gets room for all
of the rank's ``per * k`` slots), so every collective has a static size known
on the host -- no counts exchange, no ``.tolist()`` host sync -- and, on the
xGMI communicator (``XgmiAllReduce.all_to_all``, device-side epochs), the
whole MoE layer is HIP-graph capturable.  The expert id rides in an extra
column of the token row (exact in bf16 for ids <= 256); unused capacity rows
carry the null expert ``E_local``, which the grouped GEMM never computes.
The price is padding: ``ep * per * k`` rows move per rank instead of
``per * k`` -- at decode sizes the all-to-all is latency-bound, not
bandwidth-bound (prefill keeps the exact variable-size path).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import moe as M


FIXED_MAX_T = 256


def _on_xgmi(pc, nbytes: int) -> bool:
    car = pc.custom_ar
    return car is not None and pc.ep_group is pc.tp_group and car.a2a_fits(nbytes)


def _a2a(pc, send: torch.Tensor, recv: torch.Tensor, sim_fill: str = "own") -> torch.Tensor:
    """Equal-split all-to-all over the EP group: ``send`` / ``recv`` [ep, ...].
    Under tp-sim (rank 0 alone, parallel/tpsim.py) the loopback kernel moves
    the bytes, and the "peer" regions -- never written by any rank -- are then
    filled: ``"own"`` with this rank's own region (dispatch: the same routing
    statistics from every rank, so the local expert sees the row count it
    would on a real EP group; row all-gather: finite activations), ``"zero"``
    with zeros (combine: the peers' expert outputs for this rank's slots are
    not computed here -- rank 0's own block in their place would hand back
    the never-computed null-expert rows past its slot count)."""
    car = pc.custom_ar
    if send.is_cuda and send.dtype == torch.bfloat16 and _on_xgmi(pc, send.numel() * 2):
        car.all_to_all(send, recv)
        if getattr(pc, "sim", False):
            if sim_fill == "own":
                recv[1:] = recv[0:1]
            else:
                recv[1:].zero_()
        return recv
    dist.all_to_all_single(recv, send, group=pc.ep_group)
    return recv


def ep_moe_forward_fixed(moe, li: int, y: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor) -> torch.Tensor:
    """EP MoE layer with static-size collectives (see the module docstring)."""
    pc = moe.pc
    ep, r = pc.ep_size, pc.ep_rank
    T, H = y.shape
    k, El = moe.k, moe.E_local
    per = (T + ep - 1) // ep
    lo, hi = min(T, r * per), min(T, (r + 1) * per)
    n_own = hi - lo
    C = per * k                                                      # capacity per destination
    W = H + 8                                                        # row + expert-id column (16-B aligned)
    dev = y.device
    slots = torch.arange(n_own * k, device=dev)
    ids = topk_ids[lo:hi].reshape(-1).long()                         # [n_own*k] global expert ids
    dest = ids // El
    _, inv, offs = M.align(dest.to(torch.int32).view(-1, 1), ep)     # stable counting sort by destination
    pos = inv.long() - offs.long().index_select(0, dest)             # rank of the slot in its bucket
    flat = dest * C + pos                                            # its row in the [ep*C] send buffer
    send = torch.zeros(ep * C, W, dtype=y.dtype, device=dev)
    send[:, H] = float(El)                                           # null expert on unused rows
    if n_own:
        send[:, :H].index_copy_(0, flat, y.index_select(0, lo + slots // k))
        send[:, H].index_copy_(0, flat, (ids - dest * El).to(y.dtype))
    recv = _a2a(pc, send.view(ep, C * W), torch.empty(ep, C * W, dtype=y.dtype, device=dev)).view(ep * C, W)
    recv_e = recv[:, H].float().round().to(torch.int32).contiguous()
    o2, inv2, offs2 = M.align(recv_e.view(-1, 1), El + 1)            # null bucket sorts last
    xs = recv[:, :H].index_select(0, o2.long())
    # rows past offs2[El] are never computed; the grouped kernels read the offsets on the device
    ys = moe.experts(li, xs, offs2[: El + 1].contiguous(), device_offsets=True)
    out_recv = ys.index_select(0, inv2.long()).contiguous()
    back = _a2a(pc, out_recv.view(ep, C * H), torch.empty(ep, C * H, dtype=y.dtype, device=dev),
                sim_fill="zero").view(ep * C, H)
    own = y.new_zeros((per, H))
    if n_own:
        y_slots = back.index_select(0, flat)                         # (token, k) slot order
        own[:n_own] = M.combine(y_slots.contiguous(), slots.to(torch.int32), topk_w[lo:hi].contiguous(), n_own, k)
    # all-gather of the owned rows as an all-to-all of `ep` copies (one static-size collective).
    # Under tp-sim the "peer" blocks of the loopback buffer were never written:
    # they carry this rank's block instead (finite activations, like every other
    # stand-in), never the stale slots -- with those the hidden states of 7/8 of
    # the rows were garbage and the simulated runs sampled ~2 tokens each.
    gathered = _a2a(pc, own.unsqueeze(0).expand(ep, per, H).contiguous().view(ep, per * H),
                    torch.empty(ep, per * H, dtype=y.dtype, device=dev))
    return gathered.view(ep * per, H)[:T]


def ep_moe_forward(moe, li: int, y: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor) -> torch.Tensor:
    """Decode-sized batches, and every batch whose fixed-capacity dispatch fits
    the xGMI communicator (prefill included: no counts exchange, no host sync;
    the price is ``ep``-fold padded all-to-alls), take the static-size path;
    larger ones the exact variable-size RCCL path."""
    T, H = y.shape
    pc = moe.pc
    ep = pc.ep_size

    def fixed_bytes(t):
        return ep * ((t + ep - 1) // ep) * moe.k * (H + 8) * 2

    if T <= FIXED_MAX_T or (y.is_cuda and _on_xgmi(pc, fixed_bytes(T))):
        return ep_moe_forward_fixed(moe, li, y, topk_w, topk_ids)
    if y.is_cuda and _on_xgmi(pc, fixed_bytes(FIXED_MAX_T)):
        # larger than the buffer: row blocks that fit it (MoE is per token: exact)
        tc = FIXED_MAX_T
        while tc * 2 <= T and _on_xgmi(pc, fixed_bytes(tc * 2)):
            tc *= 2
        return torch.cat([ep_moe_forward_fixed(moe, li, y[a:a + tc], topk_w[a:a + tc], topk_ids[a:a + tc])
                          for a in range(0, T, tc)])
    return ep_moe_forward_var(moe, li, y, topk_w, topk_ids)


def ep_moe_forward_var(moe, li: int, y: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor) -> torch.Tensor:
    """Prefill-sized batches: exact variable-size all-to-alls (one counts
    exchange and its host sync per layer)."""
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

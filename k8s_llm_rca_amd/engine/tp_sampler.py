"""Vocab-parallel sampling across the TP ranks: one object per
TP engine rank, with the mask-table state it keeps.

Each rank holds the LM head's rows for its vocab shard, so each rank samples
its own shard: the masked Gumbel-max winner (score, global id) per row -- and,
for top-k rows, the shard's highest-scoring candidates -- is all-gathered
(a few bytes per row, on the device through the xGMI all-gather when the
group has the communicator) and combined identically on every rank, instead
of all-gathering the ``[B, vocab]`` logits.  Rank 0 (``sample_leader``)
broadcasts each step's sampling inputs, plus the grammar-mask rows the workers
have not seen, over the step channel; a worker replays them
(``sample_rows``).  The reference samples inside GPT-4's API
(``/root/reference/common/openai_generic_assistant.py:92-115``).
"""
from __future__ import annotations

from typing import Callable, List

import numpy as np
import torch

from ..ops import sampling as SMP


class VocabParallelSampler:
    def __init__(self, pc, device: torch.device, vocab: int, vocab_local: int, grt, chan,
                 to_dev: Callable[[List[np.ndarray]], List[torch.Tensor]]):
        self.pc = pc
        self.device = device
        self.vocab = vocab                # sampled vocabulary (tokenizer size)
        self.vocab_local = vocab_local    # this rank's LM-head rows
        self.grt = grt                    # grammar runtime: the mask table rank 0 broadcasts from
        self.chan = chan                  # step channel (rank 0 -> workers)
        self.to_dev = to_dev              # the engine's pinned, non-blocking multi-array upload
        self.mask_sent = 0                # rank 0: mask-table rows already broadcast to the workers
        self.wmask = None                 # every rank: device copy of the mask rows received so far

    def sample_leader(self, logits, mask_id, list_off, list_len, lists, seeds, steps, temps, topk, topp,
                      rows=None) -> torch.Tensor:
        """Rank 0: broadcast this step's sampling inputs (plus mask rows the
        workers have not seen), then sample on every rank's vocab shard."""
        import numpy as np_
        table = self.grt.masks.array() if self.grt.masks.rows else np_.zeros((0, self.grt.masks.words), np_.int32)
        new = table[self.mask_sent:]
        self.mask_sent = table.shape[0]
        B = mask_id.shape[0]
        hdr = np_.array([B, len(lists), new.shape[0], self.grt.masks.words], dtype=np_.int64)
        flat = np_.concatenate([mask_id, list_off, list_len, lists, seeds, steps, temps.view(np_.int32),
                                topk, topp.view(np_.int32), new.reshape(-1).astype(np_.int32)])
        from ..parallel.channel import SAMPLE
        rows_a = np_.asarray(rows if rows is not None else [], np_.int32)
        self.chan.send(SAMPLE, [hdr, flat, rows_a])
        return self.sample_rows(logits, hdr, flat, rows_a)

    def sample_rows(self, logits, hdr, flat, rows_a) -> torch.Tensor:
        """Every TP rank: the rows of this step's logits that sample (all when
        ``rows_a`` is empty), then the vocab-parallel sampling."""
        B, L = int(hdr[0]), int(hdr[1])
        o = 3 * B + L + 3 * B  # the payload's top_k / top_p columns (host copy: no device read)
        topk_h = flat[o:o + B]
        topp_h = flat[o + B:o + 2 * B].view(np.float32)
        if rows_a.size:
            dev, rows_d = self.to_dev([flat, rows_a])
            logits = logits.index_select(0, rows_d.long())
        else:
            dev = self.to_dev([flat])[0]
        return self._sample_shard(logits, hdr, dev, topk_h, topp_h)

    def _sample_shard(self, logits, hdr, dev, topk_h: np.ndarray, topp_h: np.ndarray) -> torch.Tensor:
        """Every TP rank: masked Gumbel-max over its vocab shard, then an
        all-gather of the [B, 2] winners (a few bytes per row instead of the
        [B, vocab] logits).  Which rows filter is read from the host copy of
        the step's payload, so no rank waits for its GPU here.

        Filtered rows: a top-k row with ``k <= CAND_K`` (any top-p) is exact
        from the ranks' candidate lists -- its whole top-k set, and so its
        nucleus and the nucleus mass, is inside them.  Any other filtered row
        (top-p without such a k, or k > CAND_K) all-gathers its logits row and
        samples it with the single-device kernel over the full vocabulary
        (same global-id noise): a nucleus of flat logits can hold thousands of
        tokens per shard, more than any candidate list."""
        import torch.distributed as dist
        B, L, nr, words = (int(x) for x in hdr)
        o = 0

        def take(n):
            nonlocal o
            t = dev[o:o + n]
            o += n
            return t

        mask_id, list_off, list_len, lists, seeds, steps = (take(B), take(B), take(B), take(L), take(B), take(B))
        temps = take(B).view(torch.float32)
        topk = take(B)
        topp = take(B).view(torch.float32)
        rows = take(nr * words).view(nr, words)
        if nr:
            self.wmask = rows.clone() if self.wmask is None else torch.cat([self.wmask, rows])
        table = self.wmask if self.wmask is not None else torch.zeros(1, words, dtype=torch.int32,
                                                                         device=self.device)
        off = self.pc.tp_rank * self.vocab_local
        filt_h = (topk_h > 0) | (topp_h < 1.0)
        cand_h = filt_h & (topk_h > 0) & (topk_h <= SMP.CAND_K)
        full_h = np.flatnonzero(filt_h & ~cand_h)
        cdev = self._gather_device()
        if cand_h.any():
            pairs, cand = SMP.sample(logits, temps, seeds, steps, mask_id, table, list_off, list_len, lists,
                                     self.vocab, vocab_off=off, pairs=True, top_k=topk, top_p=topp, candidates=True)
            # one all-gather of [B, 2 + 3 * CAND_K] per rank: the Gumbel-max winner and,
            # for top-k rows, the shard's highest-v candidates (B10 distributed top-k)
            comm = torch.cat([pairs, cand.view(B, -1)], 1).to(cdev)
        else:
            comm = SMP.sample(logits, temps, seeds, steps, mask_id, table, list_off, list_len, lists, self.vocab,
                              vocab_off=off, pairs=True).to(cdev)
        g = self._all_gather(comm)
        if cand_h.any():
            tok = SMP.combine_shards(g[:, :, :2].contiguous(), g[:, :, 2:].reshape(self.pc.tp_size, B, -1, 3),
                                     self._h2d(cand_h, g.device), topk.to(g.device), topp.to(g.device))
        else:
            tok = SMP.combine_pairs(g[:, :, :2].contiguous())
        tok = tok.to(self.device)
        if full_h.size:
            tok[self._h2d(full_h.astype(np.int64), self.device)] = self._sample_gathered(
                logits, full_h, temps, seeds, steps, mask_id, table, list_off, list_len, lists, topk, topp)
        return tok

    def _sample_gathered(self, logits, rows_h, temps, seeds, steps, mask_id, table, list_off, list_len, lists,
                         topk, topp) -> torch.Tensor:
        """Rows ``rows_h``: all-gather their logits shards and sample them over
        the whole vocabulary with the single-device kernel (every rank computes
        the same tokens)."""
        import torch.distributed as dist
        idx = self._h2d(rows_h.astype(np.int64), self.device)
        shard = logits.index_select(0, idx).float().contiguous().to(self._gather_device())
        g = self._all_gather(shard)                         # [tp, rows, vocab_local]
        full = torch.cat(list(g.unbind(0)), 1).to(self.device)  # rank r holds columns [r * vocab_local, ...)

        def pick(t):
            return t.index_select(0, idx)
        return SMP.sample(full, pick(temps), pick(seeds), pick(steps), pick(mask_id), table, pick(list_off),
                          pick(list_len), lists, self.vocab, top_k=pick(topk), top_p=pick(topp))

    @staticmethod
    def _h2d(a: np.ndarray, device) -> torch.Tensor:
        """Host array -> ``device`` without a host sync (pinned, non-blocking)."""
        t = torch.from_numpy(np.ascontiguousarray(a))
        if device.type == "cuda":
            return t.pin_memory().to(device, non_blocking=True)
        return t

    def _gather_device(self):
        """Where the sampler's per-rank winners are gathered: on the device
        through the xGMI all-to-all when the TP group has one (no host sync,
        HIP-graph capturable), else on the group's backend device."""
        car = self.pc.custom_ar
        if car is not None and self.device.type == "cuda":
            return self.device
        return self._comm_device()

    def _all_gather(self, comm: torch.Tensor) -> torch.Tensor:
        """[tp, *comm.shape]: every TP rank's ``comm``."""
        import torch.distributed as dist
        car = self.pc.custom_ar
        if car is not None and comm.is_cuda:  # device-side xGMI all-gather, any size (buffer-sized pieces)
            return car.all_gather(comm)
        parts = [torch.empty_like(comm) for _ in range(self.pc.tp_size)]
        dist.all_gather(parts, comm, group=self.pc.tp_group)
        return torch.stack(parts)

    def _comm_device(self):
        """Device of the sampling all-gather's tensors: RCCL takes device
        tensors; a gloo TP group (CPU tests, processes sharing one GPU) host ones."""
        if self.device.type != "cuda":
            return torch.device("cpu")
        import torch.distributed as dist
        return self.device if dist.get_backend(self.pc.tp_group) == "nccl" else torch.device("cpu")

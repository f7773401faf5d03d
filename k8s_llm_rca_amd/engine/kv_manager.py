"""KV cache manager: which pages every conversation thread holds, and what
happens when HBM runs short.

The engine's scheduler (``scheduler.py``) decides WHICH rows run in a step;
this object decides WHERE their KV lives.  It owns the HBM page pool
(``kv_cache.KVPool``), the optional host tier (``kv_offload.KVHostTier``) and
every policy over them:

* per-thread prefix reuse on a new run (keep the pages of the longest common
  prefix, release the rest; a page other threads share is never written);
* cross-thread prefix sharing (attach published pages, publish full ones);
* allocation with, in order of preference, swap-out of LRU idle threads to the
  host tier (and waiting for those copies), then dropping LRU idle threads
  (their next run re-prefills), then recompute PREEMPTION of younger active
  requests (``preempt_for``);
* the host tier's swap-ahead watermark and swap-in at admission.

It touches a sequence's cache fields only (``blocks``, ``bh``, ``n_cached``,
``host``, ``loading``) and the engine's stats counters; it never launches a
forward.  The reference has no cache to manage: GPT-4 re-reads each thread on
every run (``/root/reference/common/openai_generic_assistant.py:45-51``).
"""
from __future__ import annotations

from collections import Counter
from typing import Callable, Dict, List, Optional

from .kv_cache import KVPool, chain_key
from .types import Sequence


class KVCacheManager:
    def __init__(self, pool: KVPool, host=None, watermark: int = 0,
                 snapshot: Callable[[], List[Sequence]] = list, stats: Optional[Dict] = None):
        self.pool = pool
        self.host = host                # KVHostTier or None
        self.watermark = watermark      # swap ahead while free + in-flight pages are below this
        self.snapshot = snapshot        # the engine's sequences (thread-safe copy)
        self.stats = stats if stats is not None else Counter()  # standalone: counters start at 0
        self.BS = pool.block_size

    # ------------------------------------------------------------ admission
    def keep_prefix(self, s: Sequence, lcp: int) -> None:
        """A new run of ``s`` whose prompt agrees with the cached tokens on the
        first ``lcp`` (``s.n_cached`` is already ``lcp``): keep those pages and
        give up the rest.  A swapped thread starts its swap-in here."""
        BS = self.BS
        del s.bh[lcp // BS:]
        keep = (lcp + BS - 1) // BS
        if s.host is not None:  # swapped to the host tier: bring the kept pages back
            self._swap_in(s, keep)
            return
        if lcp % BS and keep <= len(s.blocks) and not self.pool.make_private(s.blocks[keep - 1]):
            # the history diverges inside a page other threads share: recompute it privately
            keep -= 1
            s.n_cached = keep * BS
        if len(s.blocks) > keep:
            self.pool.release(s.blocks[keep:])
            s.blocks = s.blocks[:keep]

    def truncate_chain(self, s: Sequence, pos: int) -> None:
        """The token at ``pos`` was rolled back: forget the chain keys from its page on."""
        del s.bh[pos // self.BS:]

    # ------------------------------------------------------------ allocation
    def ensure_blocks(self, s: Sequence, upto: int, protect: set) -> bool:
        """Pages for ``s``'s first ``upto`` tokens, making room if needed
        (never at the expense of a sequence in ``protect``)."""
        need = (upto + self.BS - 1) // self.BS - len(s.blocks)
        if need <= 0:
            return True
        if need > self.pool.free_blocks and self.host is not None:
            self._swap_make_room(need, protect)
        if need > self.pool.free_blocks:
            self.evict(need - self.pool.free_blocks, protect)
        if need > self.pool.free_blocks:
            return False
        s.blocks.extend(self.pool.alloc(need))
        return True

    def _idle(self, protect: set) -> List[Sequence]:
        """Threads without an active run that hold HBM pages, least recently used first."""
        return sorted((s for s in self.snapshot()
                       if s.req is None and s.blocks and s.id not in protect and not self.loading(s)),
                      key=lambda s: s.last_used)

    def evict(self, n_blocks: int, protect: set) -> None:
        """Drop LRU idle threads' pages (their next run re-prefills)."""
        freed = 0
        for s in self._idle(protect):
            freed += self.pool.release(s.blocks)  # pages other threads still share stay resident
            s.blocks = []
            s.bh = []
            s.n_cached = 0
            self.stats["evictions"] += 1
            if freed >= n_blocks:
                return

    def preempt_for(self, s: Sequence, upto: int, placed: set, protect: set, active: List[Sequence]) -> bool:
        """Free KV for ``s`` by preempting younger active requests (youngest
        first; not ones already placed in this step): a victim keeps its
        request and tokens, drops its pages and is re-prefilled when pages
        are free again (recompute preemption).  False if ``s`` still does not fit."""
        for v in reversed(active):
            if v is s or v.req is None or v.id in placed or not v.blocks:
                continue
            if v.req.t_submit <= s.req.t_submit:
                break  # only younger requests yield to older ones
            if self.loading(v):
                continue  # its swap-in still writes the pages
            self.pool.release(v.blocks)  # pages other threads share stay resident
            v.blocks = []
            v.bh = []
            v.n_cached = 0
            self.stats["preemptions"] += 1
            if self.ensure_blocks(s, upto, protect):
                return True
        return False

    def drop(self, s: Sequence, gone: bool = False) -> None:
        """Give up every page of ``s``, in HBM and on the host (``gone``: the
        sequence itself is released, not just its cache)."""
        if self.loading(s):
            self.host.defer_release(s.blocks, s.loading)  # the copy still writes them
            s.loading = None
        else:
            self.pool.release(s.blocks)
        s.blocks = []
        if s.host is not None:
            (self.host.free if gone else self.host.drop)(s.host)
            s.host = None
        s.bh = []
        s.n_cached = 0

    # ------------------------------------------------------------ prefix sharing
    def attach_prefix(self, s: Sequence) -> None:
        """Map the next full blocks of ``s``'s prompt onto published pages
        (at least one token is left to prefill: it produces the logits)."""
        BS = self.BS
        toks = s.tokens
        parent = s.bh[-1] if s.bh else 0
        if len(s.bh) != len(s.blocks):  # chain keys of this thread's own leading pages first
            for j in range(len(s.bh), len(s.blocks)):
                parent = chain_key(parent, toks[j * BS:(j + 1) * BS])
                s.bh.append(parent)
        n = s.n_cached
        hit = 0
        while n + BS < len(toks):
            k = chain_key(parent, toks[n:n + BS])
            b = self.pool.lookup(k)
            if b is None:
                break
            s.blocks.append(b)
            s.bh.append(k)
            parent = k
            n += BS
            hit += 1
        if hit:
            s.n_cached = n
            self.stats["prefix_hit_tokens"] += hit * BS

    def register_blocks(self, s: Sequence) -> None:
        """Publish the full pages a prefill of ``s`` has completed."""
        BS = self.BS
        toks = s.tokens
        parent = s.bh[-1] if s.bh else 0
        for j in range(len(s.bh), s.n_cached // BS):
            parent = chain_key(parent, toks[j * BS:(j + 1) * BS])
            s.bh.append(parent)
            self.pool.register(s.blocks[j], parent)

    # ------------------------------------------------------------ host tier
    def loading(self, s: Sequence) -> bool:
        """True while a swap-in of ``s``'s pages is still on the copy stream."""
        ev = s.loading
        if ev is None:
            return False
        if ev.query():
            s.loading = None
            return False
        return True

    def tick(self) -> None:
        """Once per step: release landed swap-outs and keep free + in-flight
        pages at the watermark by swapping idle threads out ahead of need."""
        if self.host is None:
            return
        t = self.host
        t.poll()
        deficit = self.watermark - self.pool.free_blocks - t.pending_blocks
        if deficit > 0:
            self._swap_out_idle(deficit, set())

    def _swap_out_idle(self, n_blocks: int, protect: set) -> int:
        """Swap LRU idle threads to the host tier until ``n_blocks`` pages are
        on their way back to the pool; returns the pages swapped."""
        t = self.host
        got = 0
        for s in self._idle(protect):
            if got >= n_blocks:
                break
            nb = len(s.blocks)
            if t.free_slots < nb:  # the host is full: give up its least recently used copies
                for v in sorted((v for v in self.snapshot() if v.host is not None and v.req is None
                                 and v.id not in protect), key=lambda v: v.last_used):
                    if t.free_slots >= nb or v.last_used > s.last_used:
                        break
                    self.drop(v)
            if t.free_slots < nb:
                break  # what is left falls to the drop path (evict)
            s.host = t.swap_out(s.blocks)
            s.blocks = []
            got += nb
            self.stats["swap_outs"] += 1
        return got

    def _swap_make_room(self, need: int, protect: set) -> None:
        """``need`` free pages now: swap idle threads out and wait for enough
        of the copies to land (the watermark makes this rare)."""
        t = self.host
        t.poll()
        short = need - self.pool.free_blocks - t.pending_blocks
        if short > 0:
            self._swap_out_idle(short, protect)
        if need > self.pool.free_blocks:
            t.wait_out(need - self.pool.free_blocks)

    def _swap_in(self, s: Sequence, keep: int) -> None:
        """Admission of a swapped thread: pages [0, keep) come back from the
        host (the run is scheduled once the copy is done), the rest are freed."""
        t = self.host
        slots, s.host = s.host, None
        keep = min(keep, len(slots))
        t.free(slots[keep:])
        s.n_cached = min(s.n_cached, keep * self.BS)
        if keep and self.ensure_blocks(s, keep * self.BS, {s.id}):
            s.loading = t.swap_in(slots[:keep], s.blocks)
            self.stats["swap_ins"] += 1
            return
        t.drop(slots[:keep])
        self.pool.release(s.blocks)
        s.blocks = []
        s.bh = []
        s.n_cached = 0

"""Host (pinned DRAM) tier under the HBM KV pool: swap idle threads out
instead of dropping them.

Every RCA pipeline keeps three assistant threads (locator, generator,
analyzer; ``/root/reference/common/openai_generic_assistant.py:45-51`` re-sends
each one to GPT-4 on every run), and only one of them runs at a time.  On a
model whose weights leave little HBM for KV (Llama-3-70B at TP=1: 141 GB of
weights, ~413k tokens of KV beside them; Mixtral with a 32k window) the idle
threads' pages are what caps the number of concurrent analyses.  Without a
host tier the pool evicts an idle thread by dropping its pages, and its next
run re-prefills the whole history (5-8k tokens: ~0.7 PFLOP at 70B).  With it:

* **swap-out** -- the LRU idle threads' pages are gathered into a contiguous
  HBM staging buffer by ``k8s_kv_stage`` (``csrc/kernels/kv_offload.hip``) and
  copied to pinned host slots by the DMA engines, both on the tier's own copy
  stream after an event of the compute stream (every write to those pages
  enqueued so far lands first).  The device pages return to the pool's free
  list only once that copy has completed (:meth:`poll`), so no later forward
  can overwrite them mid-copy.  The engine swaps ahead of need: whenever the
  free + in-flight pages fall below a watermark (``EngineConfig.kv_host_watermark``).
* **swap-in** -- when the thread's next run is admitted, the pages of its
  kept prefix are copied back (host -> staging -> fresh pool pages, same copy
  stream) and the run is scheduled once that copy's event has completed: the
  compute stream never waits on PCIe.  The bytes come back exactly as they
  left, so the run's tokens are the same as if the thread had stayed resident
  (GPU test ``test_kv_host_tier_same_tokens``).
* copy-stream order protects the host slots: a slot freed right after its
  swap-in copy was enqueued can only be overwritten by a LATER swap-out on the
  same stream.

One staging buffer serves every transfer (they are serialised on the copy
stream); a swap larger than it runs in chunks.  On CPU (tests) the same
bookkeeping runs with synchronous tensor copies.
"""
from __future__ import annotations

import ctypes
import logging
import sys
import time
import weakref
from typing import List, Optional, Tuple

import torch

from .kv_cache import KVPool

log = logging.getLogger("k8s_llm_rca_amd.engine.kv_offload")

MAX_IDS = 256  # blocks per k8s_kv_stage launch (kv_offload.hip kKvMaxIds)


def _runs(ids: List[int]) -> List[Tuple[int, int, int]]:
    """(position in ``ids``, first id, length) of each run of consecutive ids."""
    out = []
    i = 0
    while i < len(ids):
        j = i + 1
        while j < len(ids) and ids[j] == ids[j - 1] + 1:
            j += 1
        out.append((i, ids[i], j - i))
        i = j
    return out


def _unregister(host: torch.Tensor) -> None:
    from ..ops._lib import lib
    lib().k8s_host_unregister(host.data_ptr())


class KVHostTier:
    def __init__(self, pool: KVPool, host_blocks: int, staging_bytes: int = 512 << 20):
        if host_blocks < 1:
            raise ValueError("host tier needs at least one block")
        self.pool = pool
        self.device = pool.k.device
        self.cuda = self.device.type == "cuda"
        k = pool.k
        self.slab_elems = pool.nkv * pool.block_size * pool.D           # one layer's page of one block
        self.block_elems = 2 * pool.L * self.slab_elems                  # K and V, every layer
        self.block_bytes = self.block_elems * k.element_size()
        self.host_blocks = host_blocks
        t0 = time.perf_counter()
        self.host = torch.empty(host_blocks, self.block_elems, dtype=k.dtype)
        self._registered = False
        if self.cuda:  # page-locked in place (k8s_host_register): DMA-able, no power-of-two rounding
            from ..ops._lib import check, lib
            print(f"[kv_host] locking {self.host.numel() * self.host.element_size() / 1e9:.1f} GB of host memory",
                  file=sys.stderr, flush=True)
            check(lib().k8s_host_register(self.host.data_ptr(), self.host.numel() * self.host.element_size()),
                  "k8s_host_register")
            self._registered = True
            # unlocked when the tier is collected (never at interpreter exit: the OS reclaims it)
            self._fin = weakref.finalize(self, _unregister, self.host)
            self._fin.atexit = False
        self.t_pin = time.perf_counter() - t0
        self._free: List[int] = list(range(host_blocks - 1, -1, -1))
        self.chunk = max(1, min(MAX_IDS, staging_bytes // self.block_bytes))
        self._out: List[Tuple[object, List[int]]] = []  # (copy done event, device pages to release)
        self.stream = None
        self.stage = None
        if self.cuda:
            self.stream = torch.cuda.Stream(self.device)
            self.stage = torch.empty(self.chunk, self.block_elems, dtype=k.dtype, device=self.device)
        self.stats = {"out_ops": 0, "out_blocks": 0, "in_ops": 0, "in_blocks": 0, "host_dropped_blocks": 0,
                      "out_waits": 0, "out_wait_s": 0.0, "peak_host_blocks": 0}
        log.info("KV host tier: %d blocks (%.1f GB pinned in %.1f s), staging %d blocks",
                 host_blocks, host_blocks * self.block_bytes / 1e9, self.t_pin, self.chunk)

    # ------------------------------------------------------------- host slots
    @property
    def free_slots(self) -> int:
        return len(self._free)

    def alloc_slots(self, n: int) -> List[int]:
        if n > len(self._free):
            raise MemoryError(f"KV host tier exhausted: need {n}, have {len(self._free)}")
        out = sorted(self._free.pop() for _ in range(n))
        used = self.host_blocks - len(self._free)
        self.stats["peak_host_blocks"] = max(self.stats["peak_host_blocks"], used)
        return out

    def free(self, slots: List[int]) -> None:
        self._free.extend(slots)

    def drop(self, slots: List[int]) -> None:
        """A swapped thread's host copy is given up (its next run re-prefills)."""
        self.stats["host_dropped_blocks"] += len(slots)
        self.free(slots)

    # ------------------------------------------------------------- transfers
    def _stage(self, blocks: List[int], pack: bool) -> None:
        from ..ops._lib import check, lib
        ids = (ctypes.c_int * len(blocks))(*blocks)
        p = self.pool
        check(lib().k8s_kv_stage(p.k.data_ptr(), p.v.data_ptr(), self.stage.data_ptr(),
                                 self.slab_elems * p.k.element_size(), p.L, p.num_blocks, ids, len(blocks),
                                 1 if pack else 0, ctypes.c_void_p(self.stream.cuda_stream)), "k8s_kv_stage")

    def _copy(self, dst: int, src: int, n_blocks: int) -> None:
        from ..ops._lib import check, lib
        check(lib().k8s_memcpy_async(dst, src, n_blocks * self.block_bytes, ctypes.c_void_p(self.stream.cuda_stream)),
              "k8s_memcpy_async")

    def _cpu_view(self, blocks: List[int]) -> torch.Tensor:
        """[n, block_elems] image of pool pages ``blocks`` (CPU path)."""
        p = self.pool
        idx = torch.tensor(blocks, dtype=torch.long)
        kk = p.k.index_select(1, idx).transpose(0, 1).reshape(len(blocks), -1)
        vv = p.v.index_select(1, idx).transpose(0, 1).reshape(len(blocks), -1)
        return torch.cat([kk, vv], dim=1)

    def swap_out(self, blocks: List[int]) -> List[int]:
        """Copy pool pages ``blocks`` to newly allocated host slots (returned,
        in page order).  The caller gives up its references to ``blocks``
        HERE: they are released to the pool once the copy has completed."""
        slots = self.alloc_slots(len(blocks))
        self.stats["out_ops"] += 1
        self.stats["out_blocks"] += len(blocks)
        if not self.cuda:
            self.host[torch.tensor(slots)] = self._cpu_view(blocks)
            self.pool.release(blocks)
            return slots
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))
        self.stream.wait_event(ready)
        for c0 in range(0, len(blocks), self.chunk):  # gather + DMA, in order on the copy stream
            cb, cs = blocks[c0:c0 + self.chunk], slots[c0:c0 + self.chunk]
            self._stage(cb, pack=True)
            for i, s0, n in _runs(cs):
                self._copy(self.host[s0].data_ptr(), self.stage[i].data_ptr(), n)
        done = torch.cuda.Event()
        done.record(self.stream)
        self._out.append((done, list(blocks)))
        return slots

    def swap_in(self, slots: List[int], blocks: List[int]) -> Optional[object]:
        """Copy host ``slots`` into pool pages ``blocks`` (same order) and free
        the slots.  Returns the copy's completion event (None on CPU: done)."""
        assert len(slots) == len(blocks)
        self.stats["in_ops"] += 1
        self.stats["in_blocks"] += len(blocks)
        if not self.cuda:
            img = self.host[torch.tensor(slots)]
            p = self.pool
            n = len(blocks)
            half = self.block_elems // 2
            idx = torch.tensor(blocks, dtype=torch.long)
            p.k[:, idx] = img[:, :half].reshape(n, p.L, *p.k.shape[2:]).transpose(0, 1)
            p.v[:, idx] = img[:, half:].reshape(n, p.L, *p.v.shape[2:]).transpose(0, 1)
            self.free(slots)
            return None
        # the fresh pages may still be read by forwards already enqueued (pages a
        # finished thread dropped a moment ago): write them only after those
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))
        self.stream.wait_event(ready)
        for c0 in range(0, len(blocks), self.chunk):  # DMA + scatter, in order on the copy stream
            cb, cs = blocks[c0:c0 + self.chunk], slots[c0:c0 + self.chunk]
            for i, s0, n in _runs(cs):
                self._copy(self.stage[i].data_ptr(), self.host[s0].data_ptr(), n)
            self._stage(cb, pack=False)
        done = torch.cuda.Event()
        done.record(self.stream)
        self.free(slots)  # a later swap-out into them is ordered behind this copy (same stream)
        return done

    def defer_release(self, blocks: List[int], event) -> None:
        """Release pool pages once ``event`` (a swap-in writing them) completed."""
        if event is None or not blocks:
            self.pool.release(blocks)
        else:
            self._out.append((event, list(blocks)))

    # ------------------------------------------------------------- completion
    @property
    def pending_blocks(self) -> int:
        return sum(len(b) for _, b in self._out)

    def poll(self) -> int:
        """Release the pages of every completed swap-out; returns pages freed."""
        freed = 0
        keep = []
        for ev, blocks in self._out:
            if ev.query():
                freed += self.pool.release(blocks)
            else:
                keep.append((ev, blocks))
        self._out = keep
        return freed

    def wait_out(self, need: int) -> int:
        """Block until at least ``need`` pages came back (oldest copies first) or
        nothing is in flight; returns pages freed."""
        freed = self.poll()
        if freed >= need or not self._out:
            return freed
        t0 = time.perf_counter()
        self.stats["out_waits"] += 1
        while self._out and freed < need:
            ev, blocks = self._out.pop(0)
            ev.synchronize()
            freed += self.pool.release(blocks)
        self.stats["out_wait_s"] += time.perf_counter() - t0
        return freed

    def drain(self) -> None:
        """Finish every transfer (shutdown / tests)."""
        self.wait_out(1 << 62)
        if self.stream is not None:
            self.stream.synchronize()

    def close(self) -> None:
        """Finish every transfer and unlock the host buffer."""
        if self._registered:
            self.drain()
            self._fin()
            self._registered = False

    def report(self) -> dict:
        r = dict(self.stats)
        r["out_wait_s"] = round(r["out_wait_s"], 3)
        r["host_blocks"] = self.host_blocks
        r["host_gb"] = round(self.host_blocks * self.block_bytes / 1e9, 1)
        r["pin_s"] = round(self.t_pin, 1)
        return r

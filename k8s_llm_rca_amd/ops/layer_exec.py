"""Native layer executor binding (``csrc/kernels/llama_exec.hip``).

:class:`LlamaExecutor` issues the whole dense layer stack of one forward with
a single C call: per-layer weight / KV-page pointer tables are built once,
and per step only the activation buffers, the attention metadata pointers and
the GEMM kernel chosen for this step's M (:func:`..ops.linear.select_gemm`,
the same choice the Python path makes) are filled in.  Same kernels in the
same order as ``LlamaModel.forward``'s Python loop, hence bit-identical
results (``tests/test_model_gpu.py::test_layer_executor_bit_identical``).
"""
from __future__ import annotations

from ..knobs import KNOBS
import ctypes
import os
from typing import List

import torch

from . import attention as A
from . import linear as LIN
from ._lib import check, lib, ptr, scratch, stream_ptr

P = ctypes.c_void_p
I = ctypes.c_int


class GemmSel(ctypes.Structure):
    _fields_ = [("kind", I), ("cfg", I), ("splits", I), ("fuse", I)]


class LlamaStep(ctypes.Structure):
    _fields_ = [
        ("T", I), ("nd", I), ("H", I), ("nq", I), ("nkv", I), ("I", I), ("L", I), ("BS", I),
        ("eps", ctypes.c_float), ("scale", ctypes.c_float),
        ("in_norm", P), ("post_norm", P), ("wqkv", P), ("wo", P), ("wgu", P), ("wdown", P), ("kc", P), ("vc", P),
        ("residual", P), ("y", P), ("qkv", P), ("attn", P), ("obuf", P), ("gu", P), ("act", P), ("prev", P),
        ("pos", P), ("cos_sin", P), ("slots", P),
        ("d_bt", P), ("d_ctx", P), ("d_qs", P), ("d_part_o", P), ("d_part_ml", P), ("d_items", P),
        ("d_n_items_dev", P),
        ("d_bt_stride", I), ("d_S", I), ("d_n_parts", I), ("d_part_size", I), ("d_n_items", I), ("d_grid", I),
        ("p_bt", P), ("p_ctx", P), ("p_qs", P), ("tile", P * 6), ("merge", P * 4), ("pf_o", P), ("pf_ml", P),
        ("p_bt_stride", I), ("p_S", I), ("n_tiles", I), ("n_merge", I),
        ("sel", GemmSel * 4),
        ("blaslt_ws", P), ("blaslt_ws_bytes", ctypes.c_size_t), ("mid_part", P), ("grp_part", P), ("grp_offs", P),
        ("ar_id", I), ("ar_mode", I), ("ar_fuse", I), ("ar_push", I), ("nf_flags", P),
        ("res2", P), ("norm_fuse", I),
    ]


_enabled = KNOBS.layer_exec
# TP: all-reduce + residual add + RMSNorm of every row-parallel output in one launch
_fuse_ar_norm = KNOBS.tp_fused_norm
# TP: o / down projections on the stream GEMM store straight into the all-reduce's
# slots (push epilogue, csrc/kernels/allreduce.hip "push epilogue").  Off by
# default: on the tp-sim loopback the push GEMM's in-kernel publish (store acks +
# release + flag per strip, +2.5-5.4 us) costs what the consumer saves (staging,
# -2-2.5 us): 0.3-1.8 us slower per pair at 70B TP=8 decode shapes
# (tools/push_ab.py, profiles/r4/push/).  1 = push wherever the shape allows.
_tp_push = KNOBS.tp_push
# test hook: route o / down through the stream GEMM (LDS-DMA cfg 13; down split-K 2)
# wherever its shape allows, so small test models exercise both push forms
_tp_push_force = KNOBS.tp_push_force
# split-K o / down projections reduced inside the following residual add + RMSNorm
_fuse_splitk = KNOBS.fuse_splitk
# steps of <= NORM_FUSE_MAX_T rows: the input / post-attention RMSNorms computed in
# the prologue of the skinny RoPE qkv GEMM / the SwiGLU stream gate_up GEMM
# (csrc/kernels/norm_prologue.h; bit-identical, two launches fewer per layer)
_norm_fuse = KNOBS.norm_fuse
NORM_FUSE_MAX_T = 4
# (Round 3 also carried a row-chunked o / down GEMM with each chunk's
# all-reduce on a side stream, and the prefill attention on a side stream beside
# the decode attention: both measured as losses -- profiles/r3/ab/tp_overlap_*,
# profiles/r3/overlap/ -- and were retired from the executor in round 4.)
# Mixed steps as two nano-batch layer stacks on two streams (decode rows beside
# prefill rows, ops/layer_exec.py LlamaExecutor._run_nano); off by default: see
# README "Round 6" for the measurement
_nano = KNOBS.nano_batch
NANO_MIN_DECODE = 32
NANO_MIN_PREFILL = 512
_nano_serial = False  # test hook: the two stacks one after the other on the compute stream
_checked = False


def _check_abi() -> None:
    global _checked
    if not _checked:
        L = lib()
        L.k8s_llama_step_size.restype = I
        L.k8s_llama_layers.argtypes = [ctypes.POINTER(LlamaStep), P]
        L.k8s_llama_layers.restype = I
        n = L.k8s_llama_step_size()
        if n != ctypes.sizeof(LlamaStep):
            raise RuntimeError(f"LlamaStep ABI mismatch: C {n} bytes, ctypes {ctypes.sizeof(LlamaStep)}")
        _checked = True


def set_enabled(on: bool) -> None:
    global _enabled
    _enabled = on


class LlamaExecutor:
    """Bound to one dense bf16 :class:`..models.llama.LlamaModel`: TP = 1, or
    TP > 1 with the xGMI all-reduce (steps whose [T, H] all-reduce fits its
    buffer; larger prefill steps take the Python path's RCCL all-reduces)."""

    def __init__(self, model):
        _check_abi()
        self.m = model
        Ls = model.layers
        n = len(Ls)

        def table(key):
            arr = (P * n)(*[t[key].data_ptr() for t in Ls])
            return arr

        self._tabs = {k: table(k) for k in ("in_norm", "post_norm", "wqkv", "wo", "w_gu", "w_down")}
        self._kv_key = None
        self.st = LlamaStep()
        st = self.st
        cfg = model.cfg
        st.H, st.nq, st.nkv, st.I, st.L = cfg.hidden, model.nq, model.nkv, model.inter, n
        st.eps, st.scale = float(cfg.rms_eps), float(model.scale)
        st.in_norm = ctypes.addressof(self._tabs["in_norm"])
        st.post_norm = ctypes.addressof(self._tabs["post_norm"])
        st.wqkv = ctypes.addressof(self._tabs["wqkv"])
        st.wo = ctypes.addressof(self._tabs["wo"])
        st.wgu = ctypes.addressof(self._tabs["w_gu"])
        st.wdown = ctypes.addressof(self._tabs["w_down"])
        st.cos_sin = model.cos_sin.data_ptr()
        car = model.pc.custom_ar if model.pc.tp_size > 1 else None
        self._car = car
        st.ar_id = car.id if car is not None else -1
        st.ar_mode = 1
        st.ar_fuse = 0
        st.ar_push = 0
        self._side = None       # nano-batch side stream (created on first use)
        self._st_side = None
        self._side_part = None  # its split-K scratch
        self.nano_steps = 0

    @staticmethod
    def eligible(model) -> bool:
        return (_enabled and model.device.type == "cuda" and model.moe is None
                and (model.pc.tp_size == 1 or model.pc.custom_ar is not None)
                and model.dtype == torch.bfloat16 and model.D == A.HEAD_DIM and not _silu_fused_in_table(model))

    def fits(self, T: int) -> bool:
        """This step's all-reduces ([T, H] bf16) fit the xGMI buffer (always true at TP = 1)."""
        car = self._car
        if car is None:
            return True
        nb = T * self.m.cfg.hidden * 2 + (4 * T if _fuse_ar_norm else 0)  # + the fused epilogue's row sums
        return nb <= car.max_bytes and (T * self.m.cfg.hidden) % 8 == 0

    def _bind_kv(self, k_cache: torch.Tensor, v_cache: torch.Tensor) -> None:
        key = (k_cache.data_ptr(), v_cache.data_ptr(), k_cache.shape[1])
        if key == self._kv_key:
            return
        n = self.st.L
        self._kc = (P * n)(*[k_cache[li].data_ptr() for li in range(n)])
        self._vc = (P * n)(*[v_cache[li].data_ptr() for li in range(n)])
        self.st.kc = ctypes.addressof(self._kc)
        self.st.vc = ctypes.addressof(self._vc)
        self.st.BS = k_cache.shape[3]
        self._kv_key = key

    def run(self, inp, residual: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor) -> List[torch.Tensor]:
        """All layers; returns ``(prev, residual)`` for the final norm."""
        self._bind_kv(k_cache, v_cache)
        T = residual.shape[0]
        if self._nano_ok(inp, T):
            return self._run_nano(inp, residual, serial=_nano_serial)
        prev = scratch(tuple(residual.shape), residual.dtype, residual.device)
        return self._issue(self.st, inp, residual, prev, 0, T, inp.n_decode, stream_ptr(residual))

    # ------------------------------------------------------------ one layer stack
    def _issue(self, st: LlamaStep, inp, residual: torch.Tensor, prev: torch.Tensor, row0: int, T: int, nd: int,
               stream: int, side: bool = False, dry: bool = False):
        """Fill ``st`` for rows [row0, row0 + T) of the step (``nd`` decode rows
        first) and issue the layer stack on ``stream``.  ``residual`` / ``prev``
        are those rows' [T, H] buffers.  ``side``: the nano-batch side stack
        (its own split-K scratch; it must not need hipBLASLt or the grouped
        kernel, whose workspaces are single).  ``dry``: only the GEMM choices
        (returns the selection list, issues nothing)."""
        m = self.m
        H = residual.shape[1]
        dev, dt = residual.device, residual.dtype
        ld_qkv = (m.nq + 2 * m.nkv) * m.D
        H_, I_ = m.cfg.hidden, m.inter
        shapes = ((ld_qkv, H_), (H_, m.nq * m.D), (2 * I_, H_), (H_, I_))
        sels = []
        need_mid = need_grp = 0
        for i, (N, K) in enumerate(shapes):
            fused = LIN.swiglu_choice(T, N, K) if i == 2 else None  # the SwiGLU-epilogue gate_up (writes act)
            # otherwise the choice LIN.linear makes (models/llama.py's path)
            kind, cfg, splits = fused or LIN.select_gemm(T, N, K)
            if _tp_push_force and self._car is not None and i in (1, 3):
                fs = 1 if i == 1 else 2
                if LIN.stream_shape_ok(T, N, K, 13, fs):
                    kind, cfg, splits = LIN.KIND_STREAM, 13, fs
            fuse = 2 if fused else int(_fuse_splitk)
            if i == 0 and kind == LIN.KIND_SKINNY and A.skinny_rope_ok(T, N, K, m.nq, m.nkv):
                fuse = 3  # RoPE + KV write in the qkv GEMM's epilogue
            elif i == 0 and N == (m.nq + 2 * m.nkv) * m.D and LIN.rope_choice(T, N, K):
                kind, cfg, splits, fuse = LIN.KIND_BIG, LIN.BIG_PIPE, 1, 4  # gemm_big's RoPE + KV-write epilogue
            sels.append((kind, cfg, splits, fuse))
            if kind in (LIN.KIND_MID, LIN.KIND_STREAM, LIN.KIND_BIG) and splits > 1:
                need_mid = max(need_mid, splits * T * N)
            elif kind == LIN.KIND_GRP:
                need_grp = max(need_grp, splits * T * N if splits > 1 else 1)
        if dry:
            return sels
        for i, (kind, cfg, splits, fuse) in enumerate(sels):
            st.sel[i].kind, st.sel[i].cfg, st.sel[i].splits, st.sel[i].fuse = kind, cfg, splits, fuse
        y = scratch((T, H), dt, dev)
        qkv = scratch((T, ld_qkv), dt, dev)
        attn = scratch((T, m.nq * m.D), dt, dev)
        obuf = scratch((T, H), dt, dev)
        gu = scratch((T, 2 * m.inter), dt, dev)
        act = scratch((T, m.inter), dt, dev)
        st.T, st.nd = T, nd
        st.nf_flags = ptr(m.nf_flags)
        if self._car is not None:
            from ..parallel.xgmi import ONE_SHOT_MAX
            plan_for = getattr(self._car, "plan_for", None)  # the fabric-tuned plan (XgmiAllReduce.tune)
            mode, push = plan_for(T, H) if plan_for else ((1 if T * H * 2 <= ONE_SHOT_MAX else 2), False)
            st.ar_mode = mode
            # the two-shot epilogue splits each row's 16-B chunks evenly over the ranks
            st.ar_fuse = int(_fuse_ar_norm and (st.ar_mode == 1 or (H // 8) % self._car.world == 0))
            st.ar_push = int(bool(st.ar_fuse) and (_tp_push or push) and self._car.push_ok(H, T, st.ar_mode))
        st.residual, st.y, st.qkv, st.attn = residual.data_ptr(), y.data_ptr(), qkv.data_ptr(), attn.data_ptr()
        st.obuf, st.gu, st.act, st.prev = obuf.data_ptr(), gu.data_ptr(), act.data_ptr(), prev.data_ptr()
        st.pos = inp.positions.data_ptr() + 4 * row0          # int32 rows
        st.slots = ptr(inp.slots) + 4 * row0 if inp.slots is not None else None
        md = inp.meta_decode if nd > 0 else None
        if md is not None:
            st.d_bt, st.d_ctx, st.d_qs = md.block_tables.data_ptr(), md.ctx_lens.data_ptr(), md.q_start.data_ptr()
            st.d_part_o, st.d_part_ml = ptr(md.part_o), ptr(md.part_ml)
            st.d_items, st.d_n_items_dev = ptr(md.items), ptr(md.d_n_items)
            st.d_bt_stride, st.d_S = md.block_tables.stride(0), md.num_seqs
            st.d_n_parts, st.d_part_size, st.d_n_items = md.n_parts, md.part_size, md.n_items
            st.d_grid = md.grid_waves or min(A.DECODE_WAVE_SLOTS, md.n_items * m.nkv)
        else:
            st.d_bt = None
        mp = inp.meta_prefill if nd < T else None
        if mp is not None:
            if mp.n_merge and mp.pf_o is None:
                mp.pf_o, mp.pf_ml = A.prefill_workspace(m.nkv, dev, max(mp.m_slot0_end(), 1))
            st.p_bt, st.p_ctx, st.p_qs = mp.block_tables.data_ptr(), mp.ctx_lens.data_ptr(), mp.q_start.data_ptr()
            for i, t in enumerate((mp.tile_seq, mp.tile_tok0, mp.tile_len, mp.tile_kv0, mp.tile_kv1, mp.tile_slot)):
                st.tile[i] = t.data_ptr()
            for i, t in enumerate((mp.m_tok0, mp.m_len, mp.m_slot0, mp.m_np)):
                st.merge[i] = t.data_ptr()
            st.pf_o, st.pf_ml = ptr(mp.pf_o), ptr(mp.pf_ml)
            st.p_bt_stride, st.p_S, st.n_tiles, st.n_merge = mp.block_tables.stride(0), mp.num_seqs, mp.n_tiles, \
                mp.n_merge
        else:
            st.p_bt = None
        LIN.reserve_lib_workspace(dev)
        ws = LIN._blaslt_ws[dev]
        st.blaslt_ws, st.blaslt_ws_bytes = ws.data_ptr(), LIN.BLASLT_WS_BYTES
        # the same split-K buffers the Python path grows (reserved before any capture);
        # the nano-batch side stack has its own (both stacks' partials are live at once)
        if side:
            st.mid_part = self._side_scratch(dev, need_mid).data_ptr() if need_mid else None
        else:
            st.mid_part = LIN._scratch(dev, need_mid).data_ptr() if need_mid else None
        if need_grp:
            from . import moe as MO
            st.grp_part = MO._split_scratch(dev, need_grp).data_ptr()
            st.grp_offs = LIN.grp_offsets(dev, T).data_ptr()
        # fused norms (TP = 1): mirrors llama_exec.hip's nf_qkv / nf_gu conditions
        nf = 0
        if _norm_fuse and self._car is None and m.nf_flags is None and T <= NORM_FUSE_MAX_T:
            if st.sel[0].kind == LIN.KIND_SKINNY and st.sel[0].fuse == 3:
                nf |= 1
            if st.sel[2].kind == LIN.KIND_STREAM and st.sel[2].fuse == 2 and st.sel[2].cfg in (4, 8):
                nf |= 2
        st.norm_fuse = nf
        res2 = scratch((T, H), dt, dev) if nf else None
        st.res2 = ptr(res2)
        check(lib().k8s_llama_layers(ctypes.byref(st), stream), "llama_layers")
        # every fused add-norm moves the residual to the other buffer
        swaps = (st.L - 1) * (nf & 1) + st.L * ((nf >> 1) & 1)
        return prev, (res2 if swaps % 2 else residual)

    # ------------------------------------------------------------ nano-batches
    def _side_scratch(self, dev, n: int) -> torch.Tensor:
        t = self._side_part
        if t is None or t.numel() < n:
            t = self._side_part = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
        return t

    def _nano_ok(self, inp, T: int) -> bool:
        """Split this mixed step into a decode-row stack and a prefill-row stack
        on two streams (knob ``nano_batch``; TP = 1, no debug flags): the
        memory-bound decode attention and weight-streaming decode GEMMs run
        beside the compute-bound prefill GEMMs.  The decode stack must need
        neither hipBLASLt nor the grouped kernel (single workspaces)."""
        nd = inp.n_decode
        if not (_nano and self._car is None and self.m.nf_flags is None and inp.meta_decode is not None
                and inp.meta_prefill is not None and nd >= NANO_MIN_DECODE and T - nd >= NANO_MIN_PREFILL):
            return False
        res = torch.empty(0, dtype=self.m.dtype, device=self.m.device)
        sels = self._issue(self.st, inp, res.new_empty((nd, self.m.cfg.hidden)), res, 0, nd, nd, 0, dry=True)
        return all(k not in (LIN.KIND_LIB, LIN.KIND_GRP) for k, *_ in sels)

    def _run_nano(self, inp, residual: torch.Tensor, serial: bool = False):
        """Decode rows [0, nd) on a high-priority side stream, prefill rows
        [nd, T) on the compute stream, each as its own layer stack (same
        kernels as a step of only those rows); joined before the final norm.
        The two stacks share only read-only weights and disjoint KV slots.
        ``serial``: both stacks on the compute stream, one after the other
        (the reference order of the bit-identity test)."""
        T, H = residual.shape
        nd = inp.n_decode
        dev = residual.device
        main = torch.cuda.current_stream(dev)
        if self._side is None:
            self._side = torch.cuda.Stream(dev, priority=-1)
            self._st_side = LlamaStep()
            ctypes.pointer(self._st_side)[0] = self.st  # weight / KV tables, model constants
        side = self._side
        sd = self._st_side
        sd.kc, sd.vc, sd.BS = self.st.kc, self.st.vc, self.st.BS
        prev = scratch((T, H), residual.dtype, dev)
        fork = torch.cuda.Event()
        fork.record(main)
        side.wait_stream(main)
        # prefill stack first on the compute stream (it owns gemm_big's split tail)
        _, res_p = self._issue(self.st, inp, residual[nd:], prev[nd:], nd, T - nd, 0, main.cuda_stream)
        if serial:
            _, res_d = self._issue(sd, inp, residual[:nd], prev[:nd], 0, nd, nd, main.cuda_stream, side=True)
        else:
            with torch.cuda.stream(side):
                _, res_d = self._issue(sd, inp, residual[:nd], prev[:nd], 0, nd, nd, side.cuda_stream, side=True)
            residual.record_stream(side)
            prev.record_stream(side)
            main.wait_stream(side)
        self.nano_steps += 1
        # the fused-norm ping-pong needs T <= 4: never at these sizes, the stacks return their own rows
        assert res_p.data_ptr() == residual[nd:].data_ptr() and res_d.data_ptr() == residual.data_ptr()
        return prev, residual


def _silu_fused_in_table(model) -> bool:
    """The executor issues silu_mul + down GEMM; a table that fuses SwiGLU into
    the down GEMM for some M keeps the Python path (never the case today)."""
    rows = LIN.dispatch_table().get(("silu", model.cfg.hidden, model.inter))
    return bool(rows) and any(r[1] == "mid" for r in rows)

"""Token-level runtime for :mod:`.grammar` (constrained decoding).

A :class:`GrammarState` walks a compiled grammar and, at every step, tells the
engine either to *force* tokens (literal text: appended to the sequence and
prefilled in the next step -- "jump-forward", no sampling) or to *sample* one
token under a mask:

* ``("list", ids)``     explicit allow-list (choice-trie children, repeat decisions)
* ``("bitmap", row)``   a row of the device mask table (free text: every token
                        whose text has no forbidden character, plus the
                        terminator tokens once ``min_tokens`` were produced)

Choices are matched on a trie of the options' token sequences; options are
made prefix-free by appending the following literal text, so a terminal trie
node never has children.  The sampling kernel consumes the masks directly
(``csrc/kernels/sampling.hip``).
"""
from __future__ import annotations

import threading
from typing import Dict, FrozenSet, List, Optional, Sequence, Tuple

import numpy as np

from .grammar import Choice, Free, Grammar, Lit, Ref, Repeat, slot_key


class MaskTable:
    """Host registry of allow-bitmaps; the engine mirrors it to the device."""

    def __init__(self, vocab_model: int):
        self.words = (vocab_model + 31) // 32
        self.rows: List[np.ndarray] = []
        self.index: Dict[tuple, int] = {}
        self.version = 0
        self.lock = threading.Lock()

    def get(self, key: tuple, build) -> int:
        with self.lock:
            r = self.index.get(key)
            if r is None:
                bits = build()
                packed = np.packbits(bits.astype(np.uint8), bitorder="little")
                row = np.zeros(self.words * 4, dtype=np.uint8)
                row[: len(packed)] = packed
                self.rows.append(row.view(np.int32))
                r = len(self.rows) - 1
                self.index[key] = r
                self.version += 1
            return r

    def array(self) -> np.ndarray:
        return self.snapshot()[1]

    def snapshot(self):
        """(version, [rows, words] array) taken together: a version read apart
        from the rows can name a row the array does not hold yet (a mask
        registered by another thread in between), and the device mirror would
        then never be refreshed for it."""
        with self.lock:
            if not self.rows:
                return self.version, np.zeros((1, self.words), dtype=np.int32)
            return self.version, np.stack(self.rows)


class GrammarRuntime:
    """Per-tokenizer caches shared by every grammar state."""

    def __init__(self, tokenizer, vocab_model: int):
        self.tok = tokenizer
        self.vocab_model = vocab_model
        self.masks = MaskTable(vocab_model)
        self._enc_cache: Dict[str, List[int]] = {}
        self._lock = threading.Lock()
        pieces = tokenizer.pieces
        self.n_tok = len(pieces)
        self._pieces = pieces
        self._char_sets: Dict[str, np.ndarray] = {}
        specials = set(tokenizer.special.values())
        self._normal = np.array([i not in specials and pieces[i] != "" for i in range(self.n_tok)], dtype=bool)

    def encode(self, text: str) -> List[int]:
        with self._lock:
            r = self._enc_cache.get(text)
        if r is None:
            r = self.tok.encode(text)
            with self._lock:
                if len(self._enc_cache) > 100_000:
                    self._enc_cache.clear()
                self._enc_cache[text] = r
        return r

    def _free_bits(self, forbid: str) -> np.ndarray:
        b = self._char_sets.get(forbid)
        if b is None:
            ok = self._normal.copy()
            if forbid:
                fs = set(forbid)
                for i, p in enumerate(self._pieces):
                    if ok[i] and (fs.intersection(p) or "�" in p):
                        ok[i] = False
            b = ok
            self._char_sets[forbid] = b
        return b

    def free_mask(self, forbid: str, terminators: FrozenSet[int]) -> int:
        def build():
            bits = np.zeros(self.vocab_model, dtype=bool)
            bits[: self.n_tok] = self._free_bits(forbid)
            for t in terminators:
                bits[t] = True
            return bits
        return self.masks.get(("free", forbid, terminators), build)


class _Trie:
    __slots__ = ("children", "terminal", "option")

    def __init__(self):
        self.children: Dict[int, "_Trie"] = {}
        self.terminal = False
        self.option: Optional[int] = None


def _build_trie(seqs: Sequence[List[int]]) -> _Trie:
    root = _Trie()
    for oi, s in enumerate(seqs):
        n = root
        for t in s:
            n = n.children.setdefault(t, _Trie())
        n.terminal = True
        n.option = oi
    return root


# ------------------------------------------------------------- compiled ops
class _Op:
    pass


class _Force(_Op):
    __slots__ = ("text",)

    def __init__(self, text: str):
        self.text = text


class _Choice(_Op):
    __slots__ = ("options", "name", "suffix")

    def __init__(self, options: List[str], name: Optional[str], suffix: str):
        self.options = options
        self.name = name
        self.suffix = suffix  # literal text merged into every option (prefix-freeness)


class _Free(_Op):
    __slots__ = ("max_tokens", "min_tokens", "forbid", "term_text")

    def __init__(self, f: Free, term_text: Optional[str]):
        self.max_tokens = f.max_tokens
        self.min_tokens = f.min_tokens
        self.forbid = f.forbid
        self.term_text = term_text  # following literal text ('' -> end of grammar)


class _ForceIds(_Force):
    __slots__ = ("ids",)

    def __init__(self, ids: List[int]):
        super().__init__("")
        self.ids = ids


class _Repeat(_Op):
    __slots__ = ("body", "sep", "close", "min", "max", "name")

    def __init__(self, body, sep, close, mn, mx, name):
        self.body, self.sep, self.close, self.min, self.max, self.name = body, sep, close, mn, mx, name


class _Ref(_Op):
    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name


def _compile(segs: Sequence) -> List[_Op]:
    ops: List[_Op] = []
    i = 0
    segs = list(segs)
    while i < len(segs):
        s = segs[i]
        if isinstance(s, Lit):
            if ops and isinstance(ops[-1], _Force):
                ops[-1].text += s.text
            else:
                ops.append(_Force(s.text))
        elif isinstance(s, Choice):
            suffix = ""
            if i + 1 < len(segs) and isinstance(segs[i + 1], Lit):
                suffix = segs[i + 1].text
                i += 1
            ops.append(_Choice(list(s.options), s.name, suffix))
        elif isinstance(s, Free):
            term = None
            if i + 1 < len(segs) and isinstance(segs[i + 1], Lit):
                term = segs[i + 1].text
                i += 1  # the free op emits its terminator literal itself
            elif i + 1 >= len(segs):
                term = ""
            ops.append(_Free(s, term))
        elif isinstance(s, Repeat):
            ops.append(_Repeat(_compile(s.body), s.sep, s.close, s.min, s.max, s.name))
        elif isinstance(s, Ref):
            ops.append(_Ref(s.name))
        i += 1
    return ops


class GrammarState:
    """Walks one grammar for one generation.

    Protocol: call :meth:`action` -> ``("force", ids)`` | ``("sample", mask)`` |
    ``("done", None)``; after a sample call :meth:`advance` with the token.
    """

    def __init__(self, rt: GrammarRuntime, grammar: Optional[Grammar], eos_ids: Sequence[int],
                 max_tokens: int = 256, use_hints: bool = True):
        self.rt = rt
        self.eos = list(eos_ids)
        self.hints = grammar.hints if (grammar is not None and use_hints) else {}
        if grammar is None:
            grammar = Grammar([Free(max_tokens, forbid="", min_tokens=1)])
        self.ops = _compile(grammar.segments)
        # execution stack of frames: [ops, pc, suffix, repeat-ctx]
        self.stack: List[list] = [[self.ops, 0, "", None]]
        self.named: Dict[str, str] = {}
        self.sub: Optional[tuple] = None  # active sub-state
        self.n_generated = 0
        self.max_tokens = max_tokens
        self.done = False

    # ---------------------------------------------------------------- core
    def _next_op(self):
        while self.stack:
            fr = self.stack[-1]
            ops, pc, suffix, rep = fr
            if pc < len(ops):
                fr[1] += 1
                return ops[pc], suffix
            # end of a frame
            self.stack.pop()
            if rep is not None:
                op, it, psuffix = rep
                return ("repeat_next", op, it, psuffix), psuffix
        return None, ""

    def action(self):
        while True:
            if self.done:
                return ("done", None)
            if self.sub is not None:
                kind = self.sub[0]
                if kind == "choice":
                    node = self.sub[1]
                    if node.terminal:
                        self._finish_choice(self.sub)
                        continue
                    ids = list(node.children.keys())
                    return ("sample", ("list", ids))
                if kind == "free":
                    _, op, n, term_ids = self.sub
                    if n >= op.max_tokens:
                        self.sub = None
                        if op.term_text:
                            return ("force", self.rt.encode(op.term_text))
                        continue
                    terms = frozenset(term_ids[:1]) if (n >= op.min_tokens and term_ids) else frozenset()
                    return ("sample", ("bitmap", self.rt.free_mask(op.forbid, terms)))
                if kind == "decide":
                    _, op, it, suffix, seqs, node = self.sub
                    if node.terminal:
                        self.sub = None
                        cont = node.option == 0
                        self._repeat_continue(op, it, suffix, cont)
                        continue
                    return ("sample", ("list", list(node.children.keys())))
            op, suffix = self._next_op()
            if op is None:
                self.done = True
                return ("done", None)
            if isinstance(op, tuple) and op[0] == "repeat_next":
                _, rop, it, psuffix = op
                self._repeat_after_iter(rop, it, psuffix)
                continue
            if isinstance(op, _ForceIds):
                return ("force", list(op.ids))
            if isinstance(op, _Force):
                return ("force", self.rt.encode(op.text))
            if isinstance(op, _Ref):
                v = self.named.get(slot_key(op.name, suffix), self.named.get(op.name, ""))
                if v:
                    return ("force", self.rt.encode(v))
                continue
            if isinstance(op, _Choice):
                key = slot_key(op.name, suffix)
                options = op.options
                h = self.hints.get(key) if key else None
                if h is not None and h in options:
                    options = [h]
                seqs = [self.rt.encode(o + op.suffix) for o in options]
                self.sub = ("choice", _build_trie(seqs), options, key, op)
                continue
            if isinstance(op, _Free):
                if op.term_text:
                    term_ids = self.rt.encode(op.term_text)[:1]
                elif op.term_text == "":
                    term_ids = list(self.eos[:1])
                else:
                    term_ids = []
                self.sub = ("free", op, 0, term_ids)
                continue
            if isinstance(op, _Repeat):
                self._repeat_start(op, suffix)
                continue

    def _finish_choice(self, sub) -> None:
        _, node, options, key, op = sub
        if key is not None and node.option is not None:
            self.named[key] = options[node.option]
        self.sub = None

    def _repeat_start(self, op: _Repeat, suffix: str) -> None:
        self.stack.append([op.body, 0, f"{suffix}.0", (op, 0, suffix)])

    def _repeat_after_iter(self, op: _Repeat, it: int, suffix: str) -> None:
        done_iters = it + 1
        if done_iters < op.min:
            self._repeat_continue(op, it, suffix, True, emit=True)
            return
        if done_iters >= op.max:
            self._repeat_continue(op, it, suffix, False, emit=True)
            return
        key = slot_key(op.name, suffix)
        h = self.hints.get(key) if key else None
        opts = [op.sep, op.close]
        if h is not None:
            opts_idx = [0] if done_iters < int(h) else [1]
        else:
            opts_idx = [0, 1]
        seqs = [self.rt.encode(opts[i]) if i in opts_idx else None for i in range(2)]
        # a trie over the allowed decisions; option index 0 = continue, 1 = close
        root = _Trie()
        for oi, s in enumerate(seqs):
            if s is None:
                continue
            n = root
            for t in s:
                n = n.children.setdefault(t, _Trie())
            n.terminal = True
            n.option = oi
        if len(opts_idx) == 1:
            self._repeat_continue(op, it, suffix, opts_idx[0] == 0, emit=True)
            return
        self.sub = ("decide", op, it, suffix, seqs, root)

    def _repeat_continue(self, op: _Repeat, it: int, suffix: str, cont: bool, emit: bool = False) -> None:
        if cont:
            self.stack.append([op.body, 0, f"{suffix}.{it + 1}", (op, it + 1, suffix)])
        if emit:
            # emit the separator/close text before continuing
            self.stack.append([[_Force(op.sep if cont else op.close)], 0, suffix, None])

    def advance(self, token: int) -> None:
        """Consume one sampled token."""
        self.n_generated += 1
        if self.sub is None:
            raise RuntimeError("advance() without a pending sample")
        kind = self.sub[0]
        if kind == "choice":
            node = self.sub[1].children.get(token)
            if node is None:
                raise ValueError(f"token {token} not allowed by choice")
            self.sub = ("choice", node) + self.sub[2:]
        elif kind == "free":
            _, op, n, term_ids = self.sub
            if term_ids and token == term_ids[0] and n >= op.min_tokens:
                self.sub = None
                if op.term_text:
                    rest = self.rt.encode(op.term_text)[1:]
                    if rest:
                        self.stack.append([[_ForceIds(rest)], 0, "", None])
                else:
                    self.done = True
                return
            self.sub = ("free", op, n + 1, term_ids)
        elif kind == "decide":
            _, op, it, suffix, seqs, node = self.sub
            nxt = node.children.get(token)
            if nxt is None:
                raise ValueError(f"token {token} not allowed by repeat decision")
            self.sub = ("decide", op, it, suffix, seqs, nxt)
        if self.n_generated >= self.max_tokens * 4:  # runaway guard
            self.done = True


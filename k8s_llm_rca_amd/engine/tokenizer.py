"""Tokenizer + Llama-3 style chat template.

There is no network to fetch Llama-3's tokenizer, so a byte-level BPE is
trained deterministically on in-domain text (the pipeline's prompt templates,
k8s event messages, STATE JSON and Cypher from synthetic clusters with seeds
disjoint from the benchmark's) by :func:`train_tokenizer` and committed as
``k8s_llm_rca_amd/data/tokenizer.json``.  Special tokens follow Llama-3's
chat format.  The model keeps the real vocabulary size (128256 for Llama-3);
ids beyond the tokenizer are never sampled (masked).
"""
from __future__ import annotations

import functools
import os
from typing import Dict, List, Optional, Sequence

DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")
TOKENIZER_PATH = os.path.join(DATA, "tokenizer.json")

BOS = "<|begin_of_text|>"
EOS = "<|end_of_text|>"
SOH = "<|start_header_id|>"
EOH = "<|end_header_id|>"
EOT = "<|eot_id|>"
SPECIALS = [BOS, EOS, SOH, EOH, EOT]


def _corpus(n_clusters: int = 4) -> List[str]:
    from ..graph.synth import generate_cluster
    from ..pipeline import prompts as P
    from ..pipeline import generate_query as GQ
    from ..graph.schema import NATIVE_KINDS, EXTERNAL_KINDS

    texts = [P.LOCATOR_INSTRUCTIONS, P.GENERATION_TEMPLATE, P.GENERATION_LABEL_MESSAGE, P.STATE_RULE,
             P.TASK_PROMPT, P.ANALYZER_INSTRUCTIONS, P.GENERATOR_INSTRUCTIONS,
             P.build_prompt_template(NATIVE_KINDS, EXTERNAL_KINDS), P.summary_prompt(["Pod", "Secret"]),
             P.cypher_prompt("HasEvent, Event, EVENT, metadata_uid;", "msg")]
    for seed in range(1000, 1000 + n_clusters):
        c = generate_cluster(4000, 30, seed=seed)
        g = c.stategraph
        for i in range(g.num_nodes):
            p = g.node_props(i)
            for k in ("message", "spec", "status", "metadata", "path", "name2"):
                v = p.get(k)
                if isinstance(v, str):
                    texts.append(v)
        for inc in c.incidents:
            mp = "".join(f"ReferInternal, {a}, {b}, key;\n" for a, b in zip(inc.path_kinds[:-1], inc.path_kinds[1:]))
            head = ("HasEvent, Event, EVENT, metadata_uid;\n"
                    f"ReferInternal, Event, {inc.src_kind}, involvedObject_uid;\n")
            try:
                texts.append(GQ.human_generate_cypher_query(head + mp, inc.message))
            except AssertionError:
                pass
    return texts


def train_tokenizer(vocab_size: int = 32000, path: str = TOKENIZER_PATH) -> str:
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=vocab_size, special_tokens=SPECIALS, show_progress=False,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), min_frequency=2)
    tok.train_from_iterator(_corpus(), trainer=trainer)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tok.save(path)
    return path


class Tokenizer:
    def __init__(self, path: str = TOKENIZER_PATH):
        from tokenizers import Tokenizer as _T

        if not os.path.exists(path):
            train_tokenizer(path=path)
        self._tok = _T.from_file(path)
        self.vocab_size = self._tok.get_vocab_size()
        self.special: Dict[str, int] = {s: self._tok.token_to_id(s) for s in SPECIALS}
        self.bos_id = self.special[BOS]
        self.eos_id = self.special[EOS]
        self.eot_id = self.special[EOT]
        self._pieces: Optional[List[str]] = None

    def encode(self, text: str) -> List[int]:
        return self._tok.encode(text, add_special_tokens=False).ids

    def encode_batch(self, texts: Sequence[str]) -> List[List[int]]:
        return [e.ids for e in self._tok.encode_batch(list(texts), add_special_tokens=False)]

    def decode(self, ids: Sequence[int]) -> str:
        return self._tok.decode(list(ids), skip_special_tokens=True)

    @property
    def pieces(self) -> List[str]:
        """Decoded text of every token id (specials -> '')."""
        if self._pieces is None:
            out = []
            for i in range(self.vocab_size):
                out.append("" if i in self.special.values() else self._tok.decode([i]))
            self._pieces = out
        return self._pieces

    # ------------------------------------------------------- chat template
    def header(self, role: str) -> List[int]:
        return [self.special[SOH]] + self.encode(role) + [self.special[EOH]] + self.encode("\n\n")

    def message(self, role: str, content: str) -> List[int]:
        return self.header(role) + self.encode(content) + [self.eot_id]

    def system_prefix(self, instructions: str) -> List[int]:
        return [self.bos_id] + self.message("system", instructions)


@functools.lru_cache(maxsize=4)
def get_tokenizer(path: str = TOKENIZER_PATH) -> Tokenizer:
    return Tokenizer(path)

"""Deterministic synthetic tokenizer.

There is no network for real tokenizers, and weights are random, so text is
only a carrier: what the study measures is tokens and energy.  This tokenizer
is reversible for its own output and stable across processes:

* ``encode``: whitespace/punctuation pre-split, each piece hashed (blake2b)
  into the non-special id range; long words split into 4-character pieces
  (≈1.3 tokens/word on English prose, close to BPE's ≈4/3 — SURVEY §6.4);
* ``decode``: each id maps to a pronounceable synthetic piece; ids with
  ``id % 4 != 0`` start a new word, so ≈3/4 of generated tokens are words,
  matching the tokens-per-word ratio used to size ``num_predict``.

When a real ``tokenizer.json`` is available locally, ``HFTokenizer`` wraps the
``tokenizers`` library instead (no download is attempted).
"""
from __future__ import annotations

import hashlib
import math
import re
from typing import Dict, List, Optional

_SYL_C = "bdfghklmnprstvz"
_SYL_V = "aeiou"
_SPLIT = re.compile(r"\w+|[^\w\s]")

#: tokens per requested word used to size generations
TOKENS_PER_WORD = 4.0 / 3.0


def tokens_for_words(words: int) -> int:
    return int(math.ceil(TOKENS_PER_WORD * int(words)))


class SyntheticTokenizer:
    n_special = 16

    def __init__(self, vocab: int, bos_id: int = 1, eos_id: int = 2):
        self.vocab = vocab
        self.bos_id = bos_id
        self.eos_id = eos_id
        # id -> piece table, built on the first decode: detokenising a 256-row x 1,334-token step otherwise rebuilt
        # ~341k strings in Python (0.75 s, ~6 % of the step), where a real (Rust) tokenizer's decode is a table lookup
        self._table = None

    def _piece_id(self, piece: str) -> int:
        h = int.from_bytes(hashlib.blake2b(piece.encode("utf-8"), digest_size=8).digest(), "little")
        return self.n_special + h % (self.vocab - self.n_special)

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        ids = [self.bos_id] if add_bos else []
        for w in _SPLIT.findall(text):
            for i in range(0, len(w), 4):
                ids.append(self._piece_id(w[i:i + 4].lower()))
        return ids

    def piece(self, tid: int) -> str:
        return self._make_piece(tid)

    def _make_piece(self, tid: int) -> str:
        if tid < self.n_special:
            return ""
        x = tid * 2654435761 & 0xFFFFFFFF
        n = 1 + (x >> 7) % 3
        s = "".join(_SYL_C[(x >> (3 * i)) % len(_SYL_C)] + _SYL_V[(x >> (11 + 2 * i)) % len(_SYL_V)]
                    for i in range(n))
        return (" " + s) if tid % 4 else s

    def decode(self, ids: List[int]) -> str:
        import numpy as np

        if self._table is None:
            self._table = np.array([self._make_piece(t) for t in range(self.vocab)], dtype=object)
        a = np.asarray(ids, dtype=np.int64).reshape(-1)
        if a.size and (a.min() < 0 or a.max() >= self.vocab):  # out-of-vocabulary ids (tests): piece by piece
            return "".join(self._make_piece(int(t)) for t in a).lstrip()
        return "".join(self._table[a].tolist()).lstrip()

    @staticmethod
    def count_words(text: str) -> int:
        return len(text.split())


class HFTokenizer:
    """A checkpoint's ``tokenizer.json`` (``tokenizers``, Rust).  ``add_bos`` maps onto the file's own special-token
    template, as transformers does: Llama 3 and Gemma prepend their BOS there, Qwen2 adds none."""

    # the model's chat template (jinja, from tokenizer_config.json / chat_template.jinja / GGUF metadata) and the
    # special-token strings it refers to; None: prompts are used as given
    chat_template: Optional[str] = None
    special_tokens: Dict[str, str] = {}
    # prepend bos_id on encode(add_bos=True) when the tokenizer's own post-processor does not: GGUF vocabularies
    # (transformers' GGUF converters attach no BOS template) with tokenizer.ggml.add_bos_token, as llama.cpp does
    add_bos_token: bool = False

    def __init__(self, path: str, bos_id: Optional[int] = None):
        from tokenizers import Tokenizer

        self.tok = Tokenizer.from_file(path)
        self.vocab = self.tok.get_vocab_size()
        self.bos_id = bos_id
        self.special_tokens = {}

    @classmethod
    def from_tokenizer(cls, tok, bos_id: Optional[int] = None) -> "HFTokenizer":
        """Around an in-memory ``tokenizers.Tokenizer`` (a GGUF vocabulary, models/gguf.py)."""
        obj = cls.__new__(cls)
        obj.tok, obj.vocab, obj.bos_id, obj.special_tokens = tok, tok.get_vocab_size(), bos_id, {}
        return obj

    def render_chat(self, messages: List[Dict[str, str]], add_generation_prompt: bool = True) -> str:
        """``messages`` through the model's chat template, as Ollama does for ``/api/generate`` (one user message,
        unless ``raw``) and ``/api/chat``: a sandboxed jinja environment with the helpers transformers provides
        (``raise_exception``, ``strftime_now``, ``tojson``), so templates written for transformers render the same
        (tests/test_hf_checkpoint.py compares with ``apply_chat_template``)."""
        import datetime
        import json

        from jinja2.sandbox import ImmutableSandboxedEnvironment

        if not self.chat_template:
            raise ValueError("this tokenizer has no chat template")

        def raise_exception(msg):
            raise ValueError(msg)

        env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True)
        env.filters["tojson"] = lambda x, indent=None, ensure_ascii=False: json.dumps(x, indent=indent,
                                                                                      ensure_ascii=ensure_ascii)
        env.globals["raise_exception"] = raise_exception
        env.globals["strftime_now"] = lambda fmt: datetime.datetime.now().strftime(fmt)
        return env.from_string(self.chat_template).render(messages=messages,
                                                          add_generation_prompt=add_generation_prompt,
                                                          **self.special_tokens)

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        ids = self.tok.encode(text, add_special_tokens=add_bos).ids
        if add_bos and self.add_bos_token and self.bos_id is not None and (not ids or ids[0] != self.bos_id):
            ids = [int(self.bos_id)] + ids
        return ids

    def piece(self, tid: int) -> str:
        return self.tok.decode([int(tid)], skip_special_tokens=True)

    def decode(self, ids: List[int]) -> str:
        return self.tok.decode([int(t) for t in ids], skip_special_tokens=True)

    @staticmethod
    def count_words(text: str) -> int:
        return len(text.split())


class StreamDecoder:
    """Incremental detokenisation of a streamed response: the pieces ``push`` returns, followed by ``flush()`` when
    the row finishes, concatenate to ``decode(all ids)``, as Ollama's stream concatenates to its response.

    Each push decodes only a short window -- from the previous chunk's start (prefix offset) to the end -- and emits
    what that window adds beyond the previous chunk (the prefix / read offsets of TGI's and vLLM's detokenisers):
    decoding the whole sequence per push was quadratic on the scheduler thread for long streamed batches (ADVICE
    r5).  Starting the window one chunk back keeps tokenizers whose decode depends on the left context (SentencePiece
    word-boundary spaces, a stripped leading space) consistent.  A character whose bytes are split over tokens (a
    trailing U+FFFD) is held back until its last byte arrives; ``flush`` emits whatever is still held (a length
    cutoff inside a character)."""

    def __init__(self, tok):
        self.tok = tok
        self.ids: List[int] = []
        self.prefix = 0  # start of the decode window
        self.read = 0    # end of the text already emitted

    def _delta(self):
        done = self.tok.decode(self.ids[self.prefix:self.read]) if self.read > self.prefix else ""
        return done, self.tok.decode(self.ids[self.prefix:])

    def push(self, ids) -> str:
        self.ids.extend(int(t) for t in ids)
        done, text = self._delta()
        if text.endswith("\ufffd") or len(text) <= len(done):
            return ""
        self.prefix, self.read = self.read, len(self.ids)
        return text[len(done):]

    def flush(self) -> str:
        done, text = self._delta()
        self.prefix = self.read = len(self.ids)
        return text[len(done):]


def get_tokenizer(cfg, path: Optional[str] = None):
    if path:
        return HFTokenizer(path)
    return SyntheticTokenizer(cfg.vocab, cfg.bos_id, cfg.eos_id)

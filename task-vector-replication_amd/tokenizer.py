"""String ⇄ token-id helpers with TransformerLens' signatures.

The reference calls ``model.to_tokens`` / ``to_single_token`` / ``to_string``
(scratch2.py:51,64,142,182,209,298; scratch.py:126) on the GPT-NeoX BPE
tokenizer.  No tokenizer files exist offline, so the
default here is a deterministic *synthetic* tokenizer:

* pre-tokenisation with the GPT-2/NeoX regex (so " New Hampshire" is two
  tokens, "→" one, " St. Paul" three);
* every piece of the built-in task data (tasks.py) gets a fixed id 1..n in a
  fixed order — collision-free, so decoding is injective on the answer sets
  (the condition under which id comparison ≡ the reference's string
  comparison);
* other pieces hash into [n+1, V);
* ``<|endoftext|>`` is id 0 (Pythia's BOS, hard-coded by the reference at
  scratch.py:52, scratch2.py:53,121,142); ``<|123|>`` is the literal id 123
  (synthetic token-id tasks).

A real ``tokenizer.json`` can be used instead through ``HFTokenizer`` when
one is available locally.
"""
from __future__ import annotations

import zlib
from typing import Iterable, List, Sequence, Union

import regex

from . import tasks

_PRETOKENIZE = regex.compile(
    r"<\|[^|]*\|>|'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+")
_ID_LITERAL = regex.compile(r"<\|(\d+)\|>")

BOS_ID = 0
BOS_TEXT = "<|endoftext|>"


def _task_pieces() -> List[str]:
    seen, out = set(), []
    strings: List[str] = list(tasks.FUNCTION_TOKENS)
    for pairs in tasks.ALL_TASKS.values():
        for x, y in pairs:
            strings += [x, y]
    strings += tasks.us_states
    for s in strings:
        for p in _PRETOKENIZE.findall(s):
            if p not in seen and not _ID_LITERAL.fullmatch(p) and p != BOS_TEXT:
                seen.add(p)
                out.append(p)
    return out


class SyntheticTokenizer:
    def __init__(self, vocab_size: int):
        pieces = _task_pieces()
        if len(pieces) + 1 >= vocab_size:
            raise ValueError(f"vocab {vocab_size} too small for {len(pieces)} task pieces")
        self.vocab_size = vocab_size
        self._n_fixed = len(pieces) + 1
        self._to_id = {p: i + 1 for i, p in enumerate(pieces)}
        self._to_str = {i + 1: p for i, p in enumerate(pieces)}
        self._to_str[BOS_ID] = BOS_TEXT

    def piece_id(self, piece: str) -> int:
        if piece == BOS_TEXT:
            return BOS_ID
        m = _ID_LITERAL.fullmatch(piece)
        if m:
            tid = int(m.group(1))
            if not 0 <= tid < self.vocab_size:
                raise ValueError(f"token literal {piece} outside vocab {self.vocab_size}")
            return tid
        tid = self._to_id.get(piece)
        if tid is None:
            span = self.vocab_size - self._n_fixed
            tid = self._n_fixed + zlib.crc32(piece.encode()) % span
            self._to_id[piece] = tid
            self._to_str.setdefault(tid, piece)
        return tid

    def encode(self, text: str) -> List[int]:
        return [self.piece_id(p) for p in _PRETOKENIZE.findall(text)]

    def decode_one(self, tid: int) -> str:
        tid = int(tid)
        if tid in self._to_str:
            return self._to_str[tid]
        return f"<|{tid}|>"

    def decode(self, ids: Iterable[int]) -> str:
        return "".join(self.decode_one(i) for i in ids)


class HFTokenizer:
    """Wraps a local ``tokenizer.json`` (HF ``tokenizers``; Pythia's is a
    byte-level BPE with ``<|endoftext|>`` = 0) with the same API.  Decoding
    keeps special tokens, as TransformerLens' ``to_string`` does
    (``tokenizer.decode(..., clean_up_tokenization_spaces=False)``)."""

    def __init__(self, path: str):
        from tokenizers import Tokenizer
        self._tok = Tokenizer.from_file(str(path))
        self.vocab_size = self._tok.get_vocab_size()
        bos = self._tok.token_to_id(BOS_TEXT)
        if bos is not None and bos != BOS_ID:
            raise ValueError(f"{path}: {BOS_TEXT} is id {bos}; the reference hard-codes BOS = {BOS_ID} "
                             "(scratch2.py:53,121,142)")

    def encode(self, text: str) -> List[int]:
        return self._tok.encode(text, add_special_tokens=False).ids

    def decode_one(self, tid: int) -> str:
        return self._tok.decode([int(tid)], skip_special_tokens=False)

    def decode(self, ids: Iterable[int]) -> str:
        return self._tok.decode([int(i) for i in ids], skip_special_tokens=False)


TokenInput = Union[int, Sequence[int], "torch.Tensor"]  # noqa: F821


class TokenizerMixin:
    """TransformerLens-style helpers; subclasses set ``self.tokenizer`` and
    ``self.device``."""

    def to_tokens(self, text: Union[str, Sequence[str]], prepend_bos: bool = True):
        import torch
        if not isinstance(text, str):
            rows = [self.to_tokens(t, prepend_bos)[0].tolist() for t in text]
            width = max(len(r) for r in rows)
            rows = [r + [BOS_ID] * (width - len(r)) for r in rows]
            return torch.tensor(rows, dtype=torch.long, device=self.device)
        ids = ([BOS_ID] if prepend_bos else []) + self.tokenizer.encode(text)
        return torch.tensor([ids], dtype=torch.long, device=self.device)

    def to_single_token(self, text: str) -> int:
        ids = self.tokenizer.encode(text)
        # TL: assert token.numel() == 1 (HookedTransformer.to_single_token)
        assert len(ids) == 1, f"Input string: {text} is not a single token!"
        return ids[0]

    def to_string(self, tokens: TokenInput) -> Union[str, List[str]]:
        import torch
        if isinstance(tokens, torch.Tensor):
            if tokens.dim() == 0:
                return self.tokenizer.decode_one(int(tokens))
            if tokens.dim() == 1:
                return self.tokenizer.decode(tokens.tolist())
            return [self.to_string(t) for t in tokens]
        if isinstance(tokens, int):
            return self.tokenizer.decode_one(tokens)
        return self.tokenizer.decode(list(tokens))

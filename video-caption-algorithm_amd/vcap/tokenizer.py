"""GPT-2 tokenizer access without network.

The reference calls GPT2TokenizerFast.from_pretrained("gpt2") (src/models/text_decoder.py:27),
a name fetch that cannot work offline.  `load_tokenizer(dir)` builds the real byte-level BPE
tokenizer from a LOCAL vocab.json + merges.txt when a directory is given; otherwise
`IdTokenizer` keeps the same call surface (bos/eos/pad ids, __call__, decode, batch_decode)
over explicit token ids: a prompt is written "ids:464 3290 318" and captions decode to
space-joined ids.  Natural-language prompts without a vocab raise instead of guessing.
"""
from __future__ import annotations

from pathlib import Path
from types import SimpleNamespace
from typing import Iterable, List

import torch


class IdTokenizer:
    def __init__(self, eos_token_id: int = 50256):
        self.bos_token_id = self.eos_token_id = self.pad_token_id = int(eos_token_id)
        self.eos_token = self.pad_token = "<|endoftext|>"

    def encode_prompt(self, prompt: str) -> List[int]:
        """text_decoder.py:119-122: an empty prompt is [BOS]; any other string (whitespace
        included) is tokenized as given."""
        if not prompt:
            return [self.bos_token_id]
        p = prompt.strip()
        if p.startswith("ids:"):
            return [int(t) for t in p[4:].split()]
        raise ValueError("no GPT-2 vocab available offline: pass tokenizer_dir=<dir with vocab.json, merges.txt> "
                         "or a pre-tokenised prompt 'ids:<id> <id> ...'")

    def __call__(self, prompt: str, return_tensors: str = "pt"):
        return SimpleNamespace(input_ids=torch.tensor([self.encode_prompt(prompt)], dtype=torch.long))

    def decode(self, ids: Iterable[int], skip_special_tokens: bool = True) -> str:
        toks = [int(i) for i in ids]
        if skip_special_tokens:
            toks = [t for t in toks if t != self.eos_token_id]
        return " ".join(str(t) for t in toks)

    def batch_decode(self, batch, skip_special_tokens: bool = True) -> List[str]:
        return [self.decode(r, skip_special_tokens) for r in batch]


class BPETokenizer:
    """Local-file GPT-2 BPE (transformers tokenizer built from files, never fetched)."""

    def __init__(self, directory: str):
        from transformers import GPT2TokenizerFast
        d = Path(directory)
        self.tok = GPT2TokenizerFast(vocab_file=str(d / "vocab.json"), merges_file=str(d / "merges.txt"))
        if self.tok.pad_token is None:
            self.tok.pad_token = self.tok.eos_token
        self.bos_token_id, self.eos_token_id = self.tok.bos_token_id, self.tok.eos_token_id
        self.pad_token_id = self.tok.pad_token_id
        self.eos_token = self.pad_token = self.tok.eos_token

    def encode_prompt(self, prompt: str) -> List[int]:
        """text_decoder.py:119-122: [BOS] for an empty prompt, else the unmodified string's BPE ids
        (leading / trailing whitespace is tokenized, as the reference does)."""
        if not prompt:
            return [self.bos_token_id]
        if prompt.strip().startswith("ids:"):
            return [int(t) for t in prompt.strip()[4:].split()]
        return list(self.tok(prompt).input_ids)

    def __call__(self, prompt: str, return_tensors: str = "pt"):
        return SimpleNamespace(input_ids=torch.tensor([self.encode_prompt(prompt)], dtype=torch.long))

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        return self.tok.decode(list(ids), skip_special_tokens=skip_special_tokens)

    def batch_decode(self, batch, skip_special_tokens: bool = True) -> List[str]:
        return [self.decode(r, skip_special_tokens) for r in batch]


def load_tokenizer(directory: str = "", eos_token_id: int = 50256):
    if directory and (Path(directory) / "vocab.json").exists() and (Path(directory) / "merges.txt").exists():
        return BPETokenizer(directory)
    return IdTokenizer(eos_token_id)

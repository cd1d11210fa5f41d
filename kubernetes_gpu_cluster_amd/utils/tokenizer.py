"""Tokenizer resolution for offline serving.

A local HF directory with ``tokenizer.json`` uses the ``tokenizers`` fast
tokenizer (chat templates via ``transformers`` when present).  Preset models
without local files (random-init benchmarking on the network-less GPU box) get a
deterministic byte-level ``SyntheticTokenizer`` mapped into the model's vocab.
"""
from __future__ import annotations

import json
import os
from typing import Optional


class SyntheticTokenizer:
    """UTF-8 bytes -> ids [OFF, OFF+256); any other id decodes as ``<id>``."""
    OFF = 3

    def __init__(self, vocab_size: int, eos_token_id: int = 2, bos_token_id: int = 1):
        self.vocab_size = vocab_size
        self.eos_token_id = eos_token_id
        self.bos_token_id = bos_token_id

    def encode(self, text: str, add_special_tokens: bool = True) -> list[int]:
        ids = [b + self.OFF for b in text.encode("utf-8")]
        return ids or [self.OFF]

    def decode(self, ids: list[int], skip_special_tokens: bool = True) -> str:
        out = bytearray()
        parts: list[str] = []
        for i in ids:
            if self.OFF <= i < self.OFF + 256:
                out.append(i - self.OFF)
            else:
                if out:
                    parts.append(out.decode("utf-8", errors="replace"))
                    out = bytearray()
                if skip_special_tokens and i in (self.eos_token_id, self.bos_token_id):
                    continue
                parts.append(f"<{i}>")
        if out:
            parts.append(out.decode("utf-8", errors="replace"))
        return "".join(parts)

    def apply_chat_template(self, messages: list[dict], add_generation_prompt: bool = True) -> str:
        s = "".join(f"<|{m.get('role', 'user')}|>\n{m.get('content', '')}\n" for m in messages)
        return s + ("<|assistant|>\n" if add_generation_prompt else "")


class HFTokenizer:
    def __init__(self, path: str):
        from tokenizers import Tokenizer
        self.tok = Tokenizer.from_file(os.path.join(path, "tokenizer.json"))
        self.path = path
        cfg = {}
        p = os.path.join(path, "tokenizer_config.json")
        if os.path.exists(p):
            with open(p) as f:
                cfg = json.load(f)
        self.chat_template = cfg.get("chat_template")
        self._hf = None

    @property
    def vocab_size(self) -> int:
        return self.tok.get_vocab_size(with_added_tokens=True)

    def encode(self, text: str, add_special_tokens: bool = True) -> list[int]:
        return self.tok.encode(text, add_special_tokens=add_special_tokens).ids

    def decode(self, ids: list[int], skip_special_tokens: bool = True) -> str:
        return self.tok.decode(ids, skip_special_tokens=skip_special_tokens)

    def apply_chat_template(self, messages: list[dict], add_generation_prompt: bool = True) -> str:
        if self.chat_template:
            try:
                if self._hf is None:
                    from transformers import AutoTokenizer
                    self._hf = AutoTokenizer.from_pretrained(self.path)
                return self._hf.apply_chat_template(messages, tokenize=False,
                                                    add_generation_prompt=add_generation_prompt)
            except Exception:  # noqa: BLE001
                pass
        return SyntheticTokenizer.apply_chat_template(self, messages, add_generation_prompt)


def get_tokenizer(model: str, mcfg, tokenizer: Optional[str] = None,
                  allow_synthetic: bool = True):
    """``allow_synthetic=False`` (the API server with a real checkpoint) raises instead of
    falling back to the byte-level tokenizer, so a half-mounted model dir fails loudly."""
    for path in (tokenizer, model):
        if path and os.path.isfile(os.path.join(path, "tokenizer.json")):
            return HFTokenizer(path)
    if not allow_synthetic:
        raise FileNotFoundError(f"no tokenizer.json in {tokenizer or model!r}; pass --tokenizer "
                                f"DIR or --load-format dummy for a synthetic byte tokenizer")
    return SyntheticTokenizer(mcfg.vocab_size, mcfg.eos_token_id, mcfg.bos_token_id)

"""Tokenizers. No tokenizer files ship with the framework (and there is no network), so the
default is a reversible byte-level tokenizer (UTF-8 bytes -> ids 3..258, BOS=1, EOS=2); any
HuggingFace `tokenizer.json` can be used instead through `HFTokenizer` (tokenizers library)."""
from __future__ import annotations

from pathlib import Path


class ByteTokenizer:
    bos_token_id = 1
    eos_token_id = 2
    offset = 3

    def encode(self, text: str, add_bos: bool = True) -> list:
        ids = [b + self.offset for b in text.encode("utf-8")]
        return [self.bos_token_id] + ids if add_bos else ids

    def decode(self, ids) -> str:
        bs = bytes(i - self.offset for i in ids if self.offset <= i < self.offset + 256)
        return bs.decode("utf-8", errors="replace")


class HFTokenizer:
    def __init__(self, path: str | Path):
        from tokenizers import Tokenizer

        p = Path(path)
        self.tok = Tokenizer.from_file(str(p / "tokenizer.json" if p.is_dir() else p))
        self.eos_token_id = None
        self.bos_token_id = None

    def encode(self, text: str, add_bos: bool = True) -> list:
        return self.tok.encode(text).ids

    def decode(self, ids) -> str:
        return self.tok.decode(list(ids))


def load_tokenizer(path: str | None):
    return HFTokenizer(path) if path else ByteTokenizer()

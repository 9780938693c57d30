"""Tokenizers (reference lit_llama/tokenizer.py:9-89): host-side, outside the timed loop."""
import os
from pathlib import Path
from typing import Optional

import torch


class Tokenizer:
    """SentencePiece tokenizer for LLaMA (reference tokenizer.py:9-49)."""

    def __init__(self, model_path: Path) -> None:
        from sentencepiece import SentencePieceProcessor

        self.processor = SentencePieceProcessor(model_file=str(model_path))
        self.bos_id = self.processor.bos_id()
        self.eos_id = self.processor.eos_id()
        self.pad_id = self.processor.pad_id()

    @property
    def vocab_size(self) -> int:
        return self.processor.vocab_size()

    def encode(self, string: str, bos: bool = True, eos: bool = False, max_length: int = -1, pad: bool = False,
               device: Optional[torch.device] = None) -> torch.Tensor:
        return _finish(self, self.processor.encode(string), bos, eos, max_length, pad, device)

    def decode(self, tokens: torch.Tensor) -> str:
        return self.processor.decode(tokens.tolist())

    @staticmethod
    def train(input: str, destination: str, vocab_size=32000) -> None:
        from sentencepiece import SentencePieceTrainer

        model_prefix = os.path.join(destination, "tokenizer")
        SentencePieceTrainer.Train(input=input, model_prefix=model_prefix, vocab_size=vocab_size)


class HFTokenizer:
    """HF `tokenizers` JSON tokenizer with fixed BOS=1 / EOS=2 / PAD=0 (reference tokenizer.py:51-89)."""

    def __init__(self, model_path: Path) -> None:
        from tokenizers import Tokenizer as _HF

        self.processor = _HF.from_file(str(model_path))
        self.bos_id = 1
        self.eos_id = 2
        self.pad_id = 0

    @property
    def vocab_size(self) -> int:
        return self.processor.get_vocab_size()

    def encode(self, string: str, bos: bool = True, eos: bool = False, max_length: int = -1, pad: bool = False,
               device: Optional[torch.device] = None) -> torch.Tensor:
        return _finish(self, self.processor.encode(string).ids, bos, eos, max_length, pad, device)

    def decode(self, tokens: torch.Tensor) -> str:
        return self.processor.decode(tokens.tolist())


def _finish(tok, tokens, bos, eos, max_length, pad, device):
    tokens = list(tokens)
    if bos:
        tokens = [tok.bos_id] + tokens
    if eos:
        tokens = tokens + [tok.eos_id]
    if max_length > 0:
        tokens = tokens[:max_length]
    if pad and len(tokens) < max_length:
        tokens += [tok.pad_id] * (max_length - len(tokens))
    return torch.tensor(tokens, dtype=torch.int, device=device)

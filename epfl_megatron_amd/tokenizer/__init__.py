"""Tokenizers (``--tokenizer_type``)."""
from .tokenizer import build_tokenizer, vocab_size_with_padding  # noqa: F401

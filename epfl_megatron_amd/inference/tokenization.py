"""Prompt batching and detokenisation (reference ``megatron/text_generation/tokenization.py``)."""
import torch
import torch.distributed as dist

from .. import global_vars
from .communication import broadcast_int_list, broadcast_tensor, device


def _token_text(tokenizer, token):
    """Text of one token.  GPT-2 byte-level BPE decodes through its byte map
    (reference :29-33); other tokenizers detokenize the single id."""
    inner = getattr(tokenizer, "tokenizer", None)
    dec = getattr(inner, "decoder", None)
    byte_dec = getattr(inner, "byte_decoder", None)
    if isinstance(dec, dict) and isinstance(byte_dec, dict) and token in dec:
        return bytearray(byte_dec[c] for c in dec[token]).decode("utf-8", errors="replace")
    try:
        return tokenizer.detokenize([token])
    except Exception:
        return ""


def detokenize_generations(tokens_gpu_tensor, lengths_gpu_tensor, return_segments):
    tokenizer = global_vars.get_tokenizer()
    tokens = tokens_gpu_tensor.cpu().numpy().tolist()
    lengths = lengths_gpu_tensor.cpu().numpy().tolist()
    texts, segments = [], []
    for seq, n in zip(tokens, lengths):
        seq = seq[:n]
        texts.append(tokenizer.detokenize(seq))
        if return_segments:
            segments.append([_token_text(tokenizer, t) for t in seq])
    if return_segments:
        return tokens, texts, segments
    return tokens, texts


def tokenize_prompts(prompts=None, tokens_to_generate=None, add_BOS=None, rank=0):
    """Tokenise on ``rank`` and broadcast ``(tokens [b, max_len + n], lengths [b])``."""
    sizes = None
    toks = lens = None
    if dist.get_rank() == rank:
        if prompts is None or tokens_to_generate is None:
            raise AssertionError("prompts and tokens_to_generate are required on the source rank")
        toks, lens = _tokenize_prompts_and_batch(prompts, tokens_to_generate, add_BOS)
        sizes = [toks.size(0), toks.size(1)]
    sizes = broadcast_int_list(2, int_list=sizes, rank=rank).tolist()
    toks = broadcast_tensor(sizes, torch.int64, tensor=toks, rank=rank)
    lens = broadcast_tensor(sizes[0], torch.int64, tensor=lens, rank=rank)
    return toks, lens


def _tokenize_prompts_and_batch(prompts, tokens_to_generate, add_BOS):
    tokenizer = global_vars.get_tokenizer()
    bos = [tokenizer.eod] if add_BOS else []
    seqs = [bos + list(tokenizer.tokenize(p)) for p in prompts]
    lengths = [len(s) for s in seqs]
    total = max(lengths) + tokens_to_generate
    padded = [s + [tokenizer.eod] * (total - len(s)) for s in seqs]
    return (torch.tensor(padded, dtype=torch.int64, device=device()),
            torch.tensor(lengths, dtype=torch.int64, device=device()))

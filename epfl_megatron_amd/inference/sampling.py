"""Next-token sampling: greedy, top-k, top-p (nucleus), temperature
(reference ``megatron/text_generation/sampling.py``).

Semantics kept: ``top_k == 1`` is argmax; top-k and top-p are exclusive;
top-p keeps the smallest prefix of the sorted distribution whose mass
*exceeds* p, shifted by one so the token that crosses p stays eligible; the
sample is clamped to the true (unpadded) vocabulary.
"""
import torch


def modify_logits_for_top_k_filtering(logits, top_k):
    kth = torch.topk(logits, top_k, dim=-1).values[..., -1:]
    logits.masked_fill_(logits < kth, float("-inf"))


def modify_logits_for_top_p_filtering(logits, top_p):
    sorted_logits, order = torch.sort(logits, descending=True, dim=-1)
    cum = sorted_logits.softmax(dim=-1).cumsum(dim=-1)
    drop = torch.zeros_like(cum, dtype=torch.bool)
    drop[..., 1:] = cum[..., :-1] > top_p  # keep the token that crosses top_p
    logits.masked_fill_(drop.scatter(-1, order, drop), float("-inf"))


def sample(logits, top_k=0, top_p=0.0, temperature=1.0, vocab_size=None):
    """``logits`` fp32 ``[b, v]`` -> int64 ``[b]``."""
    if logits.ndim != 2:
        raise AssertionError("expected the logits to be of [b, v] shape")
    if logits.dtype != torch.float32:
        raise AssertionError("input logits should be floats")
    if top_k == 1:
        if top_p != 0.0:
            raise AssertionError("cannot set both greedy and top-p samplings")
        samples = torch.argmax(logits, dim=-1)
    else:
        logits = logits.clone()
        if temperature != 1.0:
            logits.div_(temperature)
        if top_k > 1:
            if top_p != 0.0:
                raise AssertionError("cannot set both top-k and top-p samplings")
            if top_k > logits.size(1) or (vocab_size and top_k >= vocab_size):
                raise AssertionError("top-k is larger than the vocabulary")
            modify_logits_for_top_k_filtering(logits, top_k)
        elif top_p > 0.0:
            if top_p > 1.0:
                raise AssertionError("top-p should be in (0, 1]")
            modify_logits_for_top_p_filtering(logits, top_p)
        samples = torch.multinomial(logits.softmax(dim=-1), num_samples=1).view(-1)
    if vocab_size:
        samples = samples.clamp(0, vocab_size - 1)
    return samples

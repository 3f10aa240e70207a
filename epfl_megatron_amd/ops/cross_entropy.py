"""Vocab-parallel cross-entropy.

Semantics (reference ``megatron/core/tensor_parallel/cross_entropy.py``):
per-token ``loss = log(sum_v exp(z_v)) - z_target`` over the vocab sharded
across TP ranks, computed in fp32, with the global max / target logit /
sum-of-exp combined by TP all-reduces.

MI355X design: the logits stay in their producing dtype (bf16) — the HIP
kernel (``csrc/cross_entropy.hip``) upcasts in registers, so the reference's
``[s, b, v]`` fp32 copy (1 GiB at 8k tokens x 32k vocab) is never built, and
backward recomputes ``softmax - onehot`` from the bf16 logits instead of
storing the fp32 softmax.  With TP = 1 forward is ONE pass (online max/sum);
with TP > 1 it is two passes around the RCCL all-reduces of ``[tokens]``
vectors.  Label smoothing is supported on the reference (torch) path.
"""
import torch

from ..parallel import comm, state
from ._ext import ext, use_native


def _vocab_range(part_vocab):
    rank = state.get_tensor_model_parallel_rank()
    return rank * part_vocab, (rank + 1) * part_vocab


def _tp_allreduce(t, op):
    # through parallel/comm.py: accounted ("all_reduce/tp"), race-checked,
    # looped back under the simulated-TP proxy, xGMI one-shot when registered
    if state.get_tensor_model_parallel_world_size() > 1:
        comm.all_reduce(t, group=state.get_tensor_model_parallel_group(), op=op)
    return t


class _VocabParallelCEFn(torch.autograd.Function):
    """Native path.  logits ``[..., v/tp]`` bf16/fp16/fp32, target ``[...]`` int64."""

    @staticmethod
    def forward(ctx, logits, target):
        shape = target.shape
        v = logits.shape[-1]
        z = logits.reshape(-1, v)
        if not z.is_contiguous():
            z = z.contiguous()
        tgt = target.reshape(-1).contiguous()
        start, _ = _vocab_range(v)
        tp = state.get_tensor_model_parallel_world_size()
        if tp == 1:
            loss, lse = ext().ce_fwd_fused(z, tgt)
        else:
            rmax = ext().ce_row_max(z)
            _tp_allreduce(rmax, "max")
            sumexp, tlogit = ext().ce_sumexp_target(z, tgt, rmax, start)
            _tp_allreduce(sumexp, "sum")
            _tp_allreduce(tlogit, "sum")
            lse = torch.log(sumexp) + rmax
            loss = lse - tlogit
        ctx.save_for_backward(z, tgt, lse)
        ctx.start = start
        ctx.shape = logits.shape
        return loss.view(shape)

    @staticmethod
    def backward(ctx, dloss):
        z, tgt, lse = ctx.saved_tensors
        dl = dloss.reshape(-1).float().contiguous()
        dz = ext().ce_bwd(z, tgt, lse, dl, ctx.start)
        return dz.view(ctx.shape), None


def _ce_ref(vocab_parallel_logits, target, label_smoothing=0.0):
    """fp32 torch math, TP-aware (three all-reduces like the reference)."""
    logits = vocab_parallel_logits.float()
    vmax = logits.max(dim=-1)[0]
    _tp_allreduce(vmax, "max")
    logits = logits - vmax.unsqueeze(-1)
    part_v = logits.shape[-1]
    start, end = _vocab_range(part_v)
    mask = (target < start) | (target >= end)
    local_t = (target - start).masked_fill(mask, 0)
    pred = logits.gather(-1, local_t.unsqueeze(-1)).squeeze(-1).masked_fill(mask, 0.0)
    _tp_allreduce(pred, "sum")
    sum_exp = logits.exp().sum(dim=-1)
    _tp_allreduce(sum_exp, "sum")
    loss = torch.log(sum_exp) - pred
    if label_smoothing > 0:
        vocab = part_v * state.get_tensor_model_parallel_world_size()
        smoothing = label_smoothing * vocab / (vocab - 1)
        log_probs = logits - torch.log(sum_exp).unsqueeze(-1)
        mean_lp = log_probs.sum(-1)
        _tp_allreduce(mean_lp, "sum")
        mean_lp = mean_lp / vocab
        loss = (1.0 - smoothing) * loss - smoothing * mean_lp
    return loss


class _RefCEFn(torch.autograd.Function):
    """Reference path with the reference's explicit backward (softmax - onehot)."""

    @staticmethod
    def forward(ctx, logits, target, label_smoothing):
        with torch.no_grad():
            zf = logits.float()
            vmax = zf.max(dim=-1)[0]
            _tp_allreduce(vmax, "max")
            zf = zf - vmax.unsqueeze(-1)
            part_v = zf.shape[-1]
            start, end = _vocab_range(part_v)
            mask = (target < start) | (target >= end)
            local_t = (target - start).masked_fill(mask, 0)
            pred = zf.gather(-1, local_t.unsqueeze(-1)).squeeze(-1).masked_fill(mask, 0.0)
            _tp_allreduce(pred, "sum")
            ez = zf.exp()
            sum_exp = ez.sum(-1)
            _tp_allreduce(sum_exp, "sum")
            loss = torch.log(sum_exp) - pred
            softmax = ez / sum_exp.unsqueeze(-1)
            vocab = part_v * state.get_tensor_model_parallel_world_size()
            if label_smoothing > 0:
                smoothing = label_smoothing * vocab / (vocab - 1)
                log_probs = torch.log(softmax.clamp_min(1e-30))
                mean_lp = log_probs.sum(-1)
                _tp_allreduce(mean_lp, "sum")
                loss = (1.0 - smoothing) * loss - smoothing * (mean_lp / vocab)
            ctx.save_for_backward(softmax, mask, local_t)
            ctx.label_smoothing, ctx.vocab = label_smoothing, vocab
            ctx.in_dtype = logits.dtype
        return loss

    @staticmethod
    def backward(ctx, g):
        softmax, mask, local_t = ctx.saved_tensors
        grad = softmax.clone()
        upd = (1.0 - mask.float())
        if ctx.label_smoothing > 0:
            smoothing = ctx.label_smoothing * ctx.vocab / (ctx.vocab - 1)
            grad.scatter_add_(-1, local_t.unsqueeze(-1), (-(1.0 - smoothing) * upd).unsqueeze(-1))
            grad -= smoothing / ctx.vocab
        else:
            grad.scatter_add_(-1, local_t.unsqueeze(-1), (-upd).unsqueeze(-1))
        grad.mul_(g.unsqueeze(-1))
        return grad.to(ctx.in_dtype), None, None


def vocab_parallel_cross_entropy(vocab_parallel_logits, target, label_smoothing=0.0):
    """Per-token loss (fp32) over vocab-sharded logits ``[s, b, v/tp]``."""
    if use_native(vocab_parallel_logits) and label_smoothing == 0.0:
        return _VocabParallelCEFn.apply(vocab_parallel_logits, target)
    return _RefCEFn.apply(vocab_parallel_logits, target, label_smoothing)

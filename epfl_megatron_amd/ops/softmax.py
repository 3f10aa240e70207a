"""Fused scale + mask + softmax (the non-flash attention path).

Reference kernels N1-N5 (``megatron/fused_kernels/scaled_*softmax*``) and the
dispatcher ``FusedScaleMaskSoftmax`` (``megatron/model/fused_softmax.py``).
On MI355X one HIP kernel family (``csrc/softmax.hip``) covers the three modes
(causal upper-triangular, explicit padding mask, no mask): one wave64 per row
for sk <= 1024 (four rows per workgroup, in-wave reductions), one 256-thread
workgroup per row above, the row held in registers (sk <= 8192, removing the
reference's 2048/4096 caps), 16-byte vector loads / stores, fp32
math, masked entries written as exact zeros, fully-masked rows -> 0.  A
``[1, 1, sq, sk]`` mask is read with batch stride 0 (never expanded).
Backward is ``scale * y * (dy - sum(dy * y))``.
"""
import torch

from ._ext import ext, use_native

_MODE_NONE, _MODE_CAUSAL, _MODE_MASK = 0, 1, 2
_MAX_SK = 8192


class _SoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mask, scale, mode):
        x = x.contiguous()
        y = ext().softmax_fwd(x, mask, float(scale), int(mode))
        ctx.save_for_backward(y)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return ext().softmax_bwd(dy.contiguous(), y, float(ctx.scale)), None, None, None


def attention_mask_func(scores, mask):
    return scores.masked_fill(mask, -10000.0)


class FusedScaleMaskSoftmax(torch.nn.Module):
    """scale -> mask -> softmax over the last dim of ``[b, np, sq, sk]`` scores."""

    def __init__(self, input_in_fp16, input_in_bf16, attn_mask_type, scaled_masked_softmax_fusion,
                 mask_func, softmax_in_fp32, scale):
        super().__init__()
        self.input_in_fp16 = input_in_fp16
        self.input_in_bf16 = input_in_bf16
        if input_in_fp16 and input_in_bf16:
            raise AssertionError("both fp16 and bf16 flags cannot be active at the same time.")
        self.input_in_float16 = input_in_fp16 or input_in_bf16
        self.attn_mask_type = attn_mask_type
        self.scaled_masked_softmax_fusion = scaled_masked_softmax_fusion
        self.mask_func = mask_func
        self.softmax_in_fp32 = softmax_in_fp32
        self.scale = scale
        if not (self.scale is None or softmax_in_fp32):
            raise AssertionError("softmax should be in fp32 when scaled")

    def is_kernel_available(self, x):
        b, np_, sq, sk = x.shape
        return (self.scaled_masked_softmax_fusion and use_native(x)
                and x.dtype in (torch.float16, torch.bfloat16, torch.float32)
                and 0 < sk <= _MAX_SK)

    def forward(self, x, mask):
        if x.dim() != 4:
            raise AssertionError("expected [b, np, sq, sk] scores")
        if self.is_kernel_available(x):
            scale = self.scale if self.scale is not None else 1.0
            if getattr(self.attn_mask_type, 'name', '') == 'causal':
                return _SoftmaxFn.apply(x, None, scale, _MODE_CAUSAL)
            if mask is not None:
                m = mask if mask.dtype == torch.bool else mask.bool()
                if m.dim() == 4 and m.shape[1] == 1 and m.shape[0] in (1, x.shape[0]) \
                        and tuple(m.shape[2:]) == tuple(x.shape[2:]):
                    # [b or 1, 1, sq, sk]: the kernel indexes a broadcast batch
                    return _SoftmaxFn.apply(x, m.contiguous(), scale, _MODE_MASK)
                m = m.expand(x.shape[0], 1, x.shape[2], x.shape[3]).contiguous()
                return _SoftmaxFn.apply(x, m, scale, _MODE_MASK)
            return _SoftmaxFn.apply(x, None, scale, _MODE_NONE)
        return self.forward_torch_softmax(x, mask)

    def forward_torch_softmax(self, x, mask):
        if self.input_in_float16 and self.softmax_in_fp32:
            x = x.float()
        if self.scale is not None:
            x = x * self.scale
        if getattr(self.attn_mask_type, 'name', '') == 'causal' and mask is None:
            sq, sk = x.shape[-2], x.shape[-1]
            mask = torch.ones(sq, sk, device=x.device, dtype=torch.bool).triu(1)[None, None]
        probs = torch.nn.Softmax(dim=-1)(self.mask_func(x, mask) if mask is not None else x)
        if self.input_in_float16 and self.softmax_in_fp32:
            probs = probs.half() if self.input_in_fp16 else probs.bfloat16()
        return probs

"""RMSNorm and LayerNorm.

GPU: one fused HIP kernel per direction (``csrc/norms.hip``): a row per
wave64-group, vectorised 16-byte bf16 loads, fp32 statistics, and a
two-stage deterministic reduction for the weight/bias gradients.

Numerics follow the reference:
* RMSNorm (``megatron/model/fused_layer_norm.py:125-139``): statistics in fp32,
  the normalised value is cast back to the input dtype **before** the weight
  multiply.
* LayerNorm (N6/N7, apex ``fused_layer_norm_cuda``): fp32 mean / inverse
  std, affine in fp32, one rounding to the output dtype.
"""
import torch

from ._ext import ext, use_native


def rms_norm_ref(x, weight, eps):
    xf = x.float()
    normed = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return normed.type_as(x) * weight


def layer_norm_ref(x, weight, bias, eps):
    return torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), weight.float(),
                                          None if bias is None else bias.float(), eps).type_as(x)


class _RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, eps):
        h = x.shape[-1]
        x2 = x.reshape(-1, h)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        y, rstd = ext().rmsnorm_fwd(x2, weight, eps)
        ctx.save_for_backward(x2, weight, rstd)
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, rstd = ctx.saved_tensors
        dy2 = dy.reshape(-1, x2.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx, dw = ext().rmsnorm_bwd(dy2, x2, weight, rstd)
        return dx.view(ctx.shape), dw, None


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        h = x.shape[-1]
        x2 = x.reshape(-1, h)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        y, mean, rstd = ext().layernorm_fwd(x2, weight, bias, eps)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.has_bias = bias is not None
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, mean, rstd = ctx.saved_tensors
        dy2 = dy.reshape(-1, x2.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx, dw, db = ext().layernorm_bwd(dy2, x2, weight, mean, rstd)
        return dx.view(ctx.shape), dw, (db if ctx.has_bias else None), None


def rms_norm(x, weight, eps):
    if use_native(x):
        return _RMSNormFn.apply(x, weight, eps)
    return rms_norm_ref(x, weight, eps)


def layer_norm(x, weight, bias, eps):
    if use_native(x):
        return _LayerNormFn.apply(x, weight, bias, eps)
    return layer_norm_ref(x, weight, bias, eps)


class RMSNorm(torch.nn.Module):
    """Root-mean-square norm; ``weight`` init 1 (state-dict key ``weight``)."""

    def __init__(self, dim, eps=1e-6, sequence_parallel=False):
        super().__init__()
        self.eps = eps
        self.weight = torch.nn.Parameter(torch.ones(dim))
        setattr(self.weight, "sequence_parallel", sequence_parallel)

    def forward(self, x):
        return rms_norm(x, self.weight, self.eps)


class MixedFusedLayerNorm(torch.nn.Module):
    """Affine LayerNorm (``weight`` = 1, ``bias`` = 0 at init)."""

    def __init__(self, normalized_shape, eps=1e-5, no_persist_layer_norm=True,
                 sequence_parallel=False):
        super().__init__()
        if isinstance(normalized_shape, int):
            normalized_shape = (normalized_shape,)
        self.normalized_shape = torch.Size(normalized_shape)
        self.eps = eps
        self.weight = torch.nn.Parameter(torch.ones(*normalized_shape))
        self.bias = torch.nn.Parameter(torch.zeros(*normalized_shape))
        setattr(self.weight, "sequence_parallel", sequence_parallel)
        setattr(self.bias, "sequence_parallel", sequence_parallel)

    def forward(self, x):
        return layer_norm(x, self.weight, self.bias, self.eps)

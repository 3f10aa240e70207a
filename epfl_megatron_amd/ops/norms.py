"""RMSNorm and LayerNorm.

GPU: one fused HIP kernel per direction (``csrc/norms.hip``): a row per
wave64-group, vectorised 16-byte bf16 loads, fp32 statistics, and a
two-stage deterministic reduction for the weight/bias gradients.  Under the
framework's DDP the reduction's second stage writes (or adds) the weight and
bias gradients straight into the parameters' fp32 ``main_grad`` — the
gradient-accumulation fusion the linear layers use — instead of returning a
bf16 gradient for autograd to accumulate.

Numerics follow the reference:
* RMSNorm (``megatron/model/fused_layer_norm.py:125-139``): statistics in fp32,
  the normalised value is cast back to the input dtype **before** the weight
  multiply.
* LayerNorm (N6/N7, apex ``fused_layer_norm_cuda``): fp32 mean / inverse
  std, affine in fp32, one rounding to the output dtype.
"""
import os

import torch

from ._ext import ext, use_native

# EMA_NORM_MAIN_GRAD=0: return bf16 weight gradients to autograd instead (A/B)
_FUSE_MAIN_GRAD = os.environ.get("EMA_NORM_MAIN_GRAD", "1") != "0"


def rms_norm_ref(x, weight, eps):
    xf = x.float()
    normed = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return normed.type_as(x) * weight


def layer_norm_ref(x, weight, bias, eps):
    return torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), weight.float(),
                                          None if bias is None else bias.float(), eps).type_as(x)


def _main_grad_target(param, needed):
    """(main_grad, accumulate) when ``param``'s gradient can be written by the
    norm backward kernel straight into its fp32 DDP buffer (``main_grad``, the
    gradient-accumulation fusion the linear layers use), else (None, False)."""
    if not (_FUSE_MAIN_GRAD and needed) or param is None:
        return None, False
    mg = getattr(param, "main_grad", None)
    if mg is None or not mg.is_cuda or mg.dtype != torch.float32 or not mg.is_contiguous():
        return None, False
    return mg, not getattr(param, "_mg_fresh", False)


def _main_grad_done(param):
    param._mg_fresh = False
    cb = getattr(param, "_main_grad_ready", None)
    if cb is not None:
        cb()


def _rows(t, h):
    t2 = t.reshape(-1, h)
    return t2 if t2.is_contiguous() else t2.contiguous()


class _NormResidualFn(torch.autograd.Function):
    """norm(s) and s, where s = x + res (res given) or s = x (pass-through).

    Both outputs are returned so the block can use ``s`` as its residual
    stream: in backward the residual gradient ``ds`` is added inside the norm
    backward kernel (dx = norm'(dy) + ds), which replaces the two autograd
    ``add`` kernels per block (fork of the residual, sum of its two grads).
    """

    @staticmethod
    def forward(ctx, x, res, weight, bias, eps, is_rms):
        h = x.shape[-1]
        x2 = _rows(x, h)
        r2 = None if res is None else _rows(res, h)
        if is_rms:
            y, rstd, s = ext().rmsnorm_fwd(x2, weight, eps, r2)
            ctx.save_for_backward(s, weight, rstd)
        else:
            y, mean, rstd, s = ext().layernorm_fwd(x2, weight, bias, eps, r2)
            ctx.save_for_backward(s, weight, mean, rstd)
        ctx.is_rms = is_rms
        ctx.has_res = res is not None
        ctx.has_bias = bias is not None
        ctx.shape = x.shape
        ctx.params = (weight, bias)
        s_out = s.view(x.shape) if res is not None else x
        return y.view(x.shape), s_out

    @staticmethod
    def backward(ctx, dy, ds):
        h = ctx.shape[-1]
        dy2 = _rows(dy, h)
        ds2 = None if ds is None else _rows(ds, h)
        wp, bp = ctx.params
        wacc, wa = _main_grad_target(wp, ctx.needs_input_grad[2])
        if ctx.is_rms:
            s, weight, rstd = ctx.saved_tensors
            dx, dw = ext().rmsnorm_bwd(dy2, s, weight, rstd, ds2, wacc, wa)
            db = None
        else:
            s, weight, mean, rstd = ctx.saved_tensors
            bacc, ba = _main_grad_target(bp, ctx.has_bias and ctx.needs_input_grad[3])
            dx, dw, db = ext().layernorm_bwd(dy2, s, weight, mean, rstd, ds2, wacc, bacc, wa, ba)
            if bacc is not None:
                _main_grad_done(bp)
                db = None
            if not ctx.has_bias:
                db = None
        if wacc is not None:
            _main_grad_done(wp)
            dw = None
        dx = dx.view(ctx.shape)
        return dx, (dx if ctx.has_res else None), dw, db, None, None


class _RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, eps):
        x2 = _rows(x, x.shape[-1])
        y, rstd, _ = ext().rmsnorm_fwd(x2, weight, eps)
        ctx.save_for_backward(x2, weight, rstd)
        ctx.shape = x.shape
        ctx.wparam = weight
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, rstd = ctx.saved_tensors
        wacc, wa = _main_grad_target(ctx.wparam, ctx.needs_input_grad[1])
        dx, dw = ext().rmsnorm_bwd(_rows(dy, x2.shape[-1]), x2, weight, rstd, None, wacc, wa)
        if wacc is not None:
            _main_grad_done(ctx.wparam)
            dw = None
        return dx.view(ctx.shape), dw, None


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        x2 = _rows(x, x.shape[-1])
        y, mean, rstd, _ = ext().layernorm_fwd(x2, weight, bias, eps)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.has_bias = bias is not None
        ctx.shape = x.shape
        ctx.params = (weight, bias)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, mean, rstd = ctx.saved_tensors
        wp, bp = ctx.params
        wacc, wa = _main_grad_target(wp, ctx.needs_input_grad[1])
        bacc, ba = _main_grad_target(bp, ctx.has_bias and ctx.needs_input_grad[2])
        dx, dw, db = ext().layernorm_bwd(_rows(dy, x2.shape[-1]), x2, weight, mean, rstd, None,
                                         wacc, bacc, wa, ba)
        if wacc is not None:
            _main_grad_done(wp)
            dw = None
        if bacc is not None:
            _main_grad_done(bp)
            db = None
        return dx.view(ctx.shape), dw, (db if ctx.has_bias else None), None


def rms_norm(x, weight, eps):
    if use_native(x):
        return _RMSNormFn.apply(x, weight, eps)
    return rms_norm_ref(x, weight, eps)


def layer_norm(x, weight, bias, eps):
    if use_native(x):
        return _LayerNormFn.apply(x, weight, bias, eps)
    return layer_norm_ref(x, weight, bias, eps)


def norm_residual(x, residual, weight, bias, eps, is_rms):
    """(norm(x + residual), x + residual); residual=None -> (norm(x), x)."""
    if use_native(x) and (residual is None or residual.dtype == x.dtype):
        return _NormResidualFn.apply(x, residual, weight, bias, eps, is_rms)
    s = x if residual is None else residual + x
    y = rms_norm_ref(s, weight, eps) if is_rms else layer_norm_ref(s, weight, bias, eps)
    return y, s


def _param_sync(*params):
    """Wait for the overlapped dist-opt all-gather of these parameters.

    ``DistributedDataParallel`` waits in forward pre-hooks, which fire on
    ``module(...)`` only; ``forward_residual`` is called directly by the fused
    transformer path, so it waits here (``parallel/ddp.py`` ``_param_sync_wait``)."""
    for p in params:
        wait = getattr(p, "_param_sync_wait", None) if p is not None else None
        if wait is not None:
            wait()


class RMSNorm(torch.nn.Module):
    """Root-mean-square norm; ``weight`` init 1 (state-dict key ``weight``)."""

    def __init__(self, dim, eps=1e-6, sequence_parallel=False):
        super().__init__()
        self.eps = eps
        self.weight = torch.nn.Parameter(torch.ones(dim))
        setattr(self.weight, "sequence_parallel", sequence_parallel)

    def forward(self, x):
        return rms_norm(x, self.weight, self.eps)

    def forward_residual(self, x, residual=None):
        _param_sync(self.weight)
        return norm_residual(x, residual, self.weight, None, self.eps, True)


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

    def forward_residual(self, x, residual=None):
        _param_sync(self.weight, self.bias)
        return norm_residual(x, residual, self.weight, self.bias, self.eps, False)

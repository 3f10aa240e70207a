"""GLU-family and GeLU activations.

GLU convention (reference ``megatron/model/glu_activations.py:18-21``): the
fc1 output ``[..., 2f]`` is split as ``x1, x2 = chunk(2)`` with x1 the "up"
projection (w3) and x2 the gate (w1); output ``x1 * act(x2)``.

GPU: one fused HIP kernel per direction (``csrc/activations.hip``),
16-byte vectorised, fp32 math, templated on the activation:
SwiGLU / GeGLU / ReGLU / LiGLU, and bias + tanh-GeLU (the reference's
TorchScript ``bias_gelu``) / erf-GeLU (Falcon).
"""
import torch
import torch.nn.functional as F

from ._ext import ext, use_native

_GLU_KIND = {"swiglu": 0, "geglu": 1, "reglu": 2, "liglu": 3}
_GELU_TANH, _GELU_ERF = 0, 1


def _act_ref(kind, x):
    if kind == "swiglu":
        return F.silu(x)
    if kind == "geglu":
        return F.gelu(x)
    if kind == "reglu":
        return F.relu(x)
    return x


def glu_ref(x, kind="swiglu"):
    x1, x2 = x.chunk(2, dim=-1)
    return x1 * _act_ref(kind, x2)


class _GLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kind):
        if not x.is_contiguous():
            x = x.contiguous()
        y = ext().glu_fwd(x, _GLU_KIND[kind])
        ctx.save_for_backward(x)
        ctx.kind = kind
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        if not dy.is_contiguous():
            dy = dy.contiguous()
        return ext().glu_bwd(dy, x, _GLU_KIND[ctx.kind]), None


def glu(x, kind="swiglu"):
    if use_native(x):
        return _GLUFn.apply(x, kind)
    return glu_ref(x, kind)


def swiglu(x):
    return glu(x, "swiglu")


# --- GeLU -----------------------------------------------------------------
def bias_gelu_ref(bias, y):
    x = y + bias if bias is not None else y
    return x * 0.5 * (1.0 + torch.tanh(0.79788456 * x * (1 + 0.044715 * x * x)))


def gelu_erf_ref(x):
    return F.gelu(x)


class _GeLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, approx):
        if not x.is_contiguous():
            x = x.contiguous()
        y = ext().gelu_fwd(x, bias, approx)
        ctx.save_for_backward(x, bias)
        ctx.approx = approx
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, bias = ctx.saved_tensors
        if not dy.is_contiguous():
            dy = dy.contiguous()
        dx = ext().gelu_bwd(dy, x, bias, ctx.approx)
        dbias = dx.reshape(-1, dx.shape[-1]).float().sum(0).to(bias.dtype) if ctx.has_bias else None
        return dx, dbias, None


def bias_gelu(bias, y):
    """tanh-approximate GeLU of ``y + bias`` (bias may be None)."""
    if use_native(y):
        return _GeLUFn.apply(y, bias, _GELU_TANH)
    return bias_gelu_ref(bias, y)


def gelu(x):
    """Exact (erf) GeLU — Falcon's ``F.gelu``."""
    if use_native(x):
        return _GeLUFn.apply(x, None, _GELU_ERF)
    return gelu_erf_ref(x)


# Module wrappers with the reference's names.
class _GLUModule(torch.nn.Module):
    kind = "swiglu"

    def forward(self, x):
        return glu(x, self.kind)


class SwiGLU(_GLUModule):
    kind = "swiglu"


class GEGLU(_GLUModule):
    kind = "geglu"


class ReGLU(_GLUModule):
    kind = "reglu"


class LiGLU(_GLUModule):
    kind = "liglu"


GLU_ACTIVATIONS = {"swiglu": SwiGLU(), "geglu": GEGLU(), "reglu": ReGLU(), "liglu": LiGLU()}

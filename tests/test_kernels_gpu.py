"""Numerics of every gfx950 HIP kernel against a plain PyTorch fp32 reference.

Mirrors the intent of the reference's fused-kernel tests
(megatron/fused_kernels/tests/test_fused_kernels.py) and extends them to the
kernels the reference imported from external packages (flash-attn, apex).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ext():
    from epfl_megatron_amd.ops._ext import ext
    return ext()


def _close(a, b, atol, rtol=0.0, msg=""):
    a, b = a.float(), b.float()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (~(err <= tol)).sum().item()  # NaN / inf count as off
    assert bad == 0, f"{msg}: {bad} elems off, max err {err.max().item():.3e}"


def test_extension_loaded():
    import epfl_megatron_amd._C as C
    assert hasattr(C, "flash_attn_fwd")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("H", [256, 4096, 4544, 8192])
def test_rmsnorm(dtype, H):
    from epfl_megatron_amd.ops.norms import rms_norm, rms_norm_ref
    torch.manual_seed(0)
    x = torch.randn(37, 3, H, device=DEV, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(dtype).requires_grad_()
    y = rms_norm(x, w, 1e-5)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    yr = rms_norm_ref(xr, wr, 1e-5)
    tol = 2e-2 if dtype != torch.float32 else 1e-5
    _close(y, yr, tol, 1e-2, "rmsnorm fwd")
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.float())
    _close(x.grad, xr.grad, 5e-2 if dtype != torch.float32 else 1e-4, 2e-2, "rmsnorm dx")
    _close(w.grad, wr.grad, 0.5 if dtype != torch.float32 else 1e-3, 2e-2, "rmsnorm dw")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("rows,H", [(1100, 2048), (2501, 4096), (1500, 8192)])
def test_rmsnorm_many_rows(dtype, rows, H):
    """Training-size row counts: the workgroup-per-row backward (EV = 1 / 2 / 4
    vectors per thread, odd trip counts of its two-row loop, dW partials of
    one resident wave of workgroups) against the fp32 reference."""
    from epfl_megatron_amd.ops.norms import rms_norm, rms_norm_ref
    torch.manual_seed(rows)
    x = torch.randn(rows, H, device=DEV, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(dtype).requires_grad_()
    y = rms_norm(x, w, 1e-5)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    yr = rms_norm_ref(xr, wr, 1e-5)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.float())
    _close(x.grad, xr.grad, 5e-2, 2e-2, "rmsnorm dx")
    _close(w.grad, wr.grad, 0.02 * rows ** 0.5, 2e-2, "rmsnorm dw")


@pytest.mark.parametrize("is_rms", [True, False])
@pytest.mark.parametrize("with_res", [True, False])
@pytest.mark.parametrize("rows,H", [(37, 4096), (5003, 4096), (129, 12288)])
def test_norm_residual_fused(is_rms, with_res, rows, H):
    """norm_residual(x, res) == (norm(x + res), x + res), with the residual
    gradient folded into the norm backward; rows > 2048 walks the software-
    pipelined multi-row loop of the backward kernel (odd and even trips)."""
    from epfl_megatron_amd.ops.norms import norm_residual
    torch.manual_seed(2)
    dt = torch.bfloat16
    x = torch.randn(rows, H, device=DEV, dtype=dt, requires_grad=True)
    res = torch.randn(rows, H, device=DEV, dtype=dt, requires_grad=True) if with_res else None
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(dt).requires_grad_()
    b = None if is_rms else (0.1 * torch.randn(H, device=DEV)).to(dt).requires_grad_()
    y, s = norm_residual(x, res, w, b, 1e-5, is_rms)
    xr = x.detach().float().requires_grad_()
    rr = res.detach().float().requires_grad_() if with_res else None
    wr = w.detach().float().requires_grad_()
    br = None if is_rms else b.detach().float().requires_grad_()
    sr = xr + rr if with_res else xr
    if is_rms:
        yr = sr * torch.rsqrt(sr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    else:
        yr = torch.nn.functional.layer_norm(sr, (H,), wr, br, 1e-5)
    _close(s, sr, 2e-2, 1e-2, "residual sum")
    _close(y, yr, 5e-2, 2e-2, "norm fwd")
    g1, g2 = torch.randn_like(y), torch.randn_like(s)
    ((y.float() * g1.float()).sum() + (s.float() * g2.float()).sum()).backward()
    ((yr * g1.float()).sum() + (sr * g2.float()).sum()).backward()
    _close(x.grad, xr.grad, 1e-1, 3e-2, "dx")
    if with_res:
        _close(res.grad, rr.grad, 1e-1, 3e-2, "dres")
    _close(w.grad, wr.grad, 0.02 * rows ** 0.5, 3e-2, "dw")
    if not is_rms:
        _close(b.grad, br.grad, 0.02 * rows ** 0.5, 3e-2, "db")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("H", [768, 8192])
def test_layernorm(dtype, H):
    from epfl_megatron_amd.ops.norms import layer_norm
    torch.manual_seed(1)
    x = torch.randn(65, H, device=DEV, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(dtype).requires_grad_()
    b = (0.1 * torch.randn(H, device=DEV)).to(dtype).requires_grad_()
    y = layer_norm(x, w, b, 1e-5)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (H,), wr, br, 1e-5)
    tol = 3e-2 if dtype != torch.float32 else 1e-4
    _close(y, yr, tol, 1e-2, "layernorm fwd")
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.float())
    _close(x.grad, xr.grad, tol * 3, 2e-2, "layernorm dx")
    _close(w.grad, wr.grad, 0.5 if dtype != torch.float32 else 1e-3, 2e-2, "layernorm dw")
    _close(b.grad, br.grad, 0.5 if dtype != torch.float32 else 1e-3, 2e-2, "layernorm db")


@pytest.mark.parametrize("is_rms", [True, False])
def test_norm_grad_into_main_grad(is_rms):
    """DDP gradient-accumulation fusion of the norm parameters: with a fp32
    ``main_grad`` the backward kernel writes dW (and dB) into it (fresh: =,
    then +=), fires ``_main_grad_ready`` and returns no autograd gradient."""
    from epfl_megatron_amd.ops.norms import norm_residual
    torch.manual_seed(5)
    rows, H, dt = 300, 4096, torch.bfloat16
    w = torch.nn.Parameter((1 + 0.1 * torch.randn(H, device=DEV)).to(dt))
    b = None if is_rms else torch.nn.Parameter((0.1 * torch.randn(H, device=DEV)).to(dt))
    ready = []
    for p in (w, b):
        if p is not None:
            p.main_grad = torch.full((H,), 123.0, device=DEV)
            p._mg_fresh = True
            p._main_grad_ready = (lambda q=p: ready.append(q))
    xs = [torch.randn(rows, H, device=DEV, dtype=dt, requires_grad=True) for _ in range(2)]
    gs = [torch.randn(rows, H, device=DEV, dtype=dt) for _ in range(2)]
    for x, g in zip(xs, gs):  # two micro-batches: overwrite, then accumulate
        y, _ = norm_residual(x, None, w, b, 1e-5, is_rms)
        y.backward(g)
    assert w.grad is None and (b is None or b.grad is None)
    assert len(ready) == (2 if is_rms else 4)
    wr = w.detach().float().requires_grad_()
    br = None if is_rms else b.detach().float().requires_grad_()
    for x, g in zip(xs, gs):
        xr = x.detach().float()
        if is_rms:
            yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
        else:
            yr = torch.nn.functional.layer_norm(xr, (H,), wr, br, 1e-5)
        yr.backward(g.float())
    _close(w.main_grad, wr.grad, 0.05 * rows ** 0.5, 3e-2, "dw into main_grad")
    if not is_rms:
        _close(b.main_grad, br.grad, 0.05 * rows ** 0.5, 3e-2, "db into main_grad")


@pytest.mark.parametrize("with_pos", [False, True])
def test_rope_inplace(with_pos):
    from epfl_megatron_amd.ops.rope import rope_table, rope_qkv_inplace, apply_rope_ref
    torch.manual_seed(2)
    s, b, g, r, hd = 33, 2, 4, 3, 128
    qkv = torch.randn(s, b, g, r + 2, hd, device=DEV, dtype=torch.bfloat16)
    cos, sin = rope_table(hd, 64, DEV)
    pos = None
    if with_pos:
        pos = torch.randint(0, 64, (b, s), device=DEV)
    ref = qkv.clone()
    qk = ref[:, :, :, :r + 1].reshape(s, b, g * (r + 1), hd)
    rot = apply_rope_ref(qk.float(), cos, sin, pos).view(s, b, g, r + 1, hd)
    out = qkv.clone()
    rope_qkv_inplace(out, cos, sin, pos)
    _close(out[:, :, :, :r + 1], rot, 2e-2, 1e-2, "rope q/k")
    assert torch.equal(out[:, :, :, r + 1], qkv[:, :, :, r + 1]), "v must be untouched"
    back = out.clone()
    rope_qkv_inplace(back, cos, sin, pos, inverse=True)
    _close(back, qkv, 5e-2, 2e-2, "rope inverse")


@pytest.mark.parametrize("kind", ["swiglu", "geglu", "reglu", "liglu"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_glu(kind, dtype):
    from epfl_megatron_amd.ops.activations import glu, glu_ref
    torch.manual_seed(3)
    x = torch.randn(17, 5, 2 * 688, device=DEV, dtype=dtype, requires_grad=True)
    y = glu(x, kind)
    xr = x.detach().float().requires_grad_()
    yr = glu_ref(xr, kind)
    tol = 3e-2 if dtype != torch.float32 else 1e-5
    _close(y, yr, tol, 1e-2, f"{kind} fwd")
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.float())
    _close(x.grad, xr.grad, tol * 2, 2e-2, f"{kind} bwd")


@pytest.mark.parametrize("with_bias", [False, True])
def test_gelu(with_bias):
    from epfl_megatron_amd.ops.activations import bias_gelu, bias_gelu_ref, gelu
    torch.manual_seed(4)
    x = torch.randn(64, 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    b = (0.1 * torch.randn(1024, device=DEV)).bfloat16().requires_grad_() if with_bias else None
    y = bias_gelu(b, x)
    xr = x.detach().float().requires_grad_()
    br = b.detach().float().requires_grad_() if with_bias else None
    yr = bias_gelu_ref(br, xr)
    _close(y, yr, 3e-2, 1e-2, "bias_gelu fwd")
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.float())
    _close(x.grad, xr.grad, 5e-2, 2e-2, "bias_gelu dx")
    if with_bias:
        _close(b.grad, br.grad, 0.5, 2e-2, "bias_gelu db")
    x2 = x.detach().clone().requires_grad_()
    y2 = gelu(x2)
    _close(y2, torch.nn.functional.gelu(x2.float()), 3e-2, 1e-2, "erf gelu")


@pytest.mark.parametrize("V", [512, 32000])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_cross_entropy(V, dtype):
    from epfl_megatron_amd.ops.cross_entropy import vocab_parallel_cross_entropy
    torch.manual_seed(5)
    z = (3 * torch.randn(9, 4, V, device=DEV)).to(dtype).requires_grad_()
    t = torch.randint(0, V, (9, 4), device=DEV)
    loss = vocab_parallel_cross_entropy(z, t)
    zr = z.detach().float().requires_grad_()
    lr = torch.nn.functional.cross_entropy(zr.view(-1, V), t.view(-1), reduction="none").view(9, 4)
    _close(loss, lr, 1e-3, 1e-4, "ce fwd")
    g = torch.rand_like(loss)
    loss.backward(g)
    lr.backward(g)
    _close(z.grad, zr.grad, 1e-2 if dtype != torch.float32 else 1e-6, 1e-2, "ce bwd")


def test_cross_entropy_tp_pieces():
    """Two-pass (TP>1) kernels combined on one device == full-vocab CE."""
    torch.manual_seed(6)
    e = _ext()
    V, rows = 1024, 50
    z = torch.randn(rows, V, device=DEV, dtype=torch.bfloat16)
    t = torch.randint(0, V, (rows,), device=DEV)
    halves = z.chunk(2, dim=1)
    m = torch.stack([e.ce_row_max(h.contiguous()) for h in halves]).max(0)[0]
    se, tl = 0, 0
    for i, h in enumerate(halves):
        a, b = e.ce_sumexp_target(h.contiguous(), t, m, i * (V // 2))
        se, tl = se + a, tl + b
    loss = torch.log(se) + m - tl
    ref = torch.nn.functional.cross_entropy(z.float(), t, reduction="none")
    _close(loss, ref, 1e-3, 1e-4, "ce tp")


@pytest.mark.parametrize("mode", ["causal", "mask", "mask_bcast", "none"])
@pytest.mark.parametrize("sk,dtype", [
    (16, torch.bfloat16), (60, torch.bfloat16), (128, torch.bfloat16), (520, torch.float16),
    (1000, torch.bfloat16), (1024, torch.float32), (2000, torch.bfloat16),
    (4096, torch.bfloat16), (3000, torch.float32)])
def test_fused_softmax(mode, sk, dtype):
    """csrc/softmax.hip: wave-per-row (sk <= 1024) and workgroup-per-row forms,
    16-B vector and element-wise row lengths, bf16 / fp16 / fp32, causal /
    explicit / batch-broadcast ([1, 1, sq, sk], read with stride 0) masks,
    vs the fp32 torch softmax (reference megatron/model/fused_softmax.py)."""
    from epfl_megatron_amd.ops.softmax import _SoftmaxFn, FusedScaleMaskSoftmax
    torch.manual_seed(7)
    b, np_, sq = 2, 3, min(sk, 512) if mode == "causal" else 37
    if mode == "causal":
        sk = sq
    x = torch.randn(b, np_, sq, sk, device=DEV, dtype=dtype, requires_grad=True)
    scale = 0.5
    xf = x.detach().float() * scale
    mask = None
    if mode == "causal":
        m = torch.ones(sq, sk, device=DEV, dtype=torch.bool).triu(1)
        ref = torch.softmax(xf.masked_fill(m, float("-inf")), -1)
        y = _SoftmaxFn.apply(x, None, scale, 1)
    elif mode in ("mask", "mask_bcast"):
        mb = b if mode == "mask" else 1
        mask = torch.rand(mb, 1, sq, sk, device=DEV) < 0.3
        mask[..., 3, :] = True  # a fully masked row -> zeros
        ref = torch.softmax(xf.masked_fill(mask, -10000.0), -1)
        ref[..., 3, :] = 0.0
        y = _SoftmaxFn.apply(x, mask, scale, 2)
        if mode == "mask_bcast":  # the module path takes the broadcast mask as is
            mod = FusedScaleMaskSoftmax(dtype == torch.float16, dtype == torch.bfloat16, None,
                                        True, None, True, scale)
            _close(mod(x.detach(), mask), ref, 1e-2, 2e-2, "softmax module bcast")
    else:
        ref = torch.softmax(xf, -1)
        y = _SoftmaxFn.apply(x, None, scale, 0)
    tol = (1e-5, 1e-4) if dtype == torch.float32 else (1e-2, 2e-2)
    _close(y, ref, *tol, f"softmax {mode}")
    g = torch.randn_like(y)
    y.backward(g)
    yf = ref
    dref = scale * yf * (g.float() - (g.float() * yf).sum(-1, keepdim=True))
    tol = (1e-4, 1e-3) if dtype == torch.float32 else (2e-2, 3e-2)
    _close(x.grad, dref, *tol, f"softmax bwd {mode}")


def test_flat_adam_and_norm():
    from epfl_megatron_amd.ops import optim_kernels as K
    torch.manual_seed(8)
    n = 300000
    segs = [(0, 0, 100000, 0, True), (100032, 100032, 150000, 1, False),
            (250048, 250048, 49952, 0, True)]
    total = 300000
    plan = K.ChunkPlan(segs, DEV)
    grad = torch.randn(total, device=DEV)
    master = torch.randn(total, device=DEV)
    m = torch.randn(total, device=DEV).abs() * 0.1
    v = torch.randn(total, device=DEV).abs() * 0.1
    model = master.to(torch.bfloat16)
    refs = [t.clone().cpu() for t in (master, m, v)]
    nsq = K.grad_norm_sq(grad, plan)
    cpu_plan = K.ChunkPlan(segs, "cpu")
    nsq_ref = K.grad_norm_sq(grad.cpu(), cpu_plan)
    assert abs(nsq.item() - nsq_ref.item()) / nsq_ref.item() < 1e-5
    K.adam_step(master, model, grad, m, v, plan, [1e-3, 2e-3], [0.1, 0.0], 0.9, 0.95, 1e-8, 3, 0.7)
    mr, m_r, v_r = refs
    model_ref = torch.zeros(total, dtype=torch.bfloat16)
    K.adam_step(mr, model_ref, grad.cpu(), m_r, v_r, cpu_plan, [1e-3, 2e-3], [0.1, 0.0], 0.9, 0.95,
                1e-8, 3, 0.7)
    _close(master.cpu(), mr, 1e-6, 1e-5, "adam master")
    _close(m.cpu(), m_r, 1e-6, 1e-5, "adam m")
    _close(v.cpu(), v_r, 1e-6, 1e-5, "adam v")
    for lo, hi in ((0, 100000), (100032, 250032), (250048, 300000)):
        _close(model[lo:hi].cpu(), mr[lo:hi].to(torch.bfloat16), 1e-2, 1e-2, "adam model write")


def _attn_case(b, s, nq, nkv, hd, dtype, causal, seed=0):
    from epfl_megatron_amd.ops.attention import flash_attn_func, attention_ref
    torch.manual_seed(seed)
    q = torch.randn(b, s, nq, hd, device=DEV, dtype=dtype, requires_grad=True)
    k = torch.randn(b, s, nkv, hd, device=DEV, dtype=dtype, requires_grad=True)
    v = torch.randn(b, s, nkv, hd, device=DEV, dtype=dtype, requires_grad=True)
    o = flash_attn_func(q, k, v, causal=causal)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = attention_ref(qr, kr, vr, causal=causal)
    _close(o, orf, 2e-2, 2e-2, "flash fwd")
    g = torch.randn_like(o)
    o.backward(g)
    orf.backward(g.float())
    _close(q.grad, qr.grad, 5e-2, 5e-2, "flash dq")
    _close(k.grad, kr.grad, 5e-2, 5e-2, "flash dk")
    _close(v.grad, vr.grad, 5e-2, 5e-2, "flash dv")


@pytest.mark.parametrize("hd", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("nq,nkv", [(4, 4), (8, 2), (4, 1)])
def test_flash_attention(hd, causal, nq, nkv):
    _attn_case(2, 256, nq, nkv, hd, torch.bfloat16, causal)


@pytest.mark.parametrize("s", [1, 77, 200, 1000])
def test_flash_attention_odd_lengths(s):
    _attn_case(1, s, 4, 2, 128, torch.bfloat16, True, seed=s)


def test_flash_attention_seq4096():
    """The Llama-2 native context (BASELINE config #3 shape per head)."""
    _attn_case(1, 4096, 4, 4, 128, torch.bfloat16, True, seed=41)


@pytest.mark.parametrize("nq,nkv", [(71, 1), (32, 2), (16, 8)])
def test_flash_attention_falcon_shapes(nq, nkv):
    """Falcon head layouts at head_dim 64: 7B MQA (71/1), 40B-TP4-like (32/2), GQA (16/8)."""
    _attn_case(1, 320, nq, nkv, 64, torch.bfloat16, True, seed=nq)


@pytest.mark.parametrize("b,s,nq,nkv,causal", [
    (4, 1024, 32, 32, True),   # Llama-2-7B training shape: 512 blocks of 256 rows
    (4, 1024, 32, 32, False),
    (2, 2048, 32, 8, True),    # GQA at seq 2k
    (1, 4000, 64, 64, True),   # partial last tile, 16 x 64 blocks
])
def test_flash_attention_8wave(b, s, nq, nkv, causal):
    """Grids large enough for the 8-wave forward and dQ kernels (3-slot K/V
    ring, flash_attn_fwd.hip / flash_attn_bwd.hip)."""
    assert (s + 255) // 256 * nq * b >= 512  # flash_attn_waves() picks 8
    _attn_case(b, s, nq, nkv, 128, torch.bfloat16, causal, seed=s + nkv)


def test_flash_attention_causal_pairing():
    """A causal grid of exactly two 4-wave blocks per CU (one TP rank of a
    TP-sharded model: 16 heads x 4096 tokens = 512 blocks of 128 rows) runs its
    second round of query blocks lightest-first (kernels.h pair_ncu): == the
    fp32 reference, and bitwise equal to the plain heavy-first order."""
    from epfl_megatron_amd.ops.attention import flash_attn_func
    C = _ext()
    b, s, nq, hd = 1, 4096, 16, 128
    assert (s + 255) // 256 * nq * b < 512  # flash_attn_waves() picks 4
    _attn_case(b, s, nq, nq, hd, torch.bfloat16, True, seed=17)
    torch.manual_seed(18)
    q, k, v = (torch.randn(b, s, nq, hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)
               for _ in range(3))
    g = torch.randn(b, s, nq, hd, device=DEV, dtype=torch.bfloat16)
    outs = []
    for on in (True, False):
        C.fa_set_pairing(on)
        try:
            for t in (q, k, v):
                t.grad = None
            o = flash_attn_func(q, k, v, causal=True)
            o.backward(g)
            outs.append([o.detach().clone()] + [t.grad.clone() for t in (q, k, v)])
        finally:
            C.fa_set_pairing(True)
    for a, bb, name in zip(outs[0], outs[1], ("o", "dq", "dk", "dv")):
        assert torch.equal(a, bb), name


@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_split_key_forward(causal):
    """One TP rank of Llama-2-70B at TP = 8 (8 query heads on one KV head, 4096
    tokens: 256 blocks of 128 rows, one per CU) runs the split-key forward
    (fa_fwd_k KV2: two 4-wave halves of the key range, merged through LDS) and
    the split-key dQ (fa_bwd_dq2_k KV2, partials added through LDS): fwd + bwd
    == the fp32 reference; the forward with it on and off close to each other.
    Smaller head_dim-128 grids in this file run it too."""
    from epfl_megatron_amd.ops.attention import flash_attn_func, attention_ref
    C = _ext()
    b, s, nq, nkv, hd = 1, 4096, 8, 1, 128
    _attn_case(b, s, nq, nkv, hd, torch.bfloat16, causal, seed=21)
    torch.manual_seed(22)
    q = torch.randn(b, s, nq, hd, device=DEV, dtype=torch.bfloat16)
    k, v = (torch.randn(b, s, nkv, hd, device=DEV, dtype=torch.bfloat16) for _ in range(2))
    ref = attention_ref(q.float(), k.float(), v.float(), causal=causal)
    outs = []
    for on in (True, False):
        C.fa_set_kv2(on)
        try:
            outs.append(flash_attn_func(q, k, v, causal=causal))
        finally:
            C.fa_set_kv2(True)
    _close(outs[0], ref, 2e-2, 2e-2, "split-key forward")
    _close(outs[1], ref, 2e-2, 2e-2, "4-wave forward")
    _close(outs[0], outs[1], 2e-2, 2e-2, "split-key vs 4-wave")


def test_flash_attention_running_max_jump():
    """Online-softmax rescale branch forced: one key row aligned with one query
    row so that row's running max jumps by a large margin at a late tile
    (rule: a rare data-dependent branch needs its own test)."""
    from epfl_megatron_amd.ops.attention import flash_attn_func, attention_ref
    torch.manual_seed(77)
    b, s, nq, hd = 1, 640, 2, 128
    q = torch.randn(b, s, nq, hd, device=DEV)
    k = torch.randn(b, s, nq, hd, device=DEV) * 0.3
    v = torch.randn(b, s, nq, hd, device=DEV)
    for row, key in ((600, 530), (301, 300), (64, 5)):
        k[:, key] = q[:, row] * 2.0  # score(row, key) >> every other score of the row
    q, k, v = (t.to(torch.bfloat16) for t in (q, k, v))
    o = flash_attn_func(q, k, v, causal=True)
    orf = attention_ref(q.float(), k.float(), v.float(), causal=True)
    _close(o, orf, 2e-2, 2e-2, "flash fwd with running-max jumps")


def test_flash_attention_fp16():
    _attn_case(1, 192, 4, 4, 128, torch.float16, True)


@pytest.mark.parametrize("s,b,ng,r,hd,with_pos", [
    (300, 2, 2, 3, 128, False),   # GQA, dK/dV split over query heads (reduce-kernel epilogue)
    (4096, 1, 2, 1, 128, False),  # Llama-2 native context, MHA (dK/dV kernel epilogue)
    (257, 2, 1, 8, 64, True),     # Falcon-like MQA, head_dim 64, explicit position ids
])
def test_flash_attention_qkvpacked_rope(s, b, ng, r, hd, with_pos):
    """The training path: fused GQA QKV + RoPE fused into FA (k-only rotation
    pass, Q rotated in the forward kernel, R^T on dQ/dK in the backward
    epilogues), fwd and bwd against the fp32 CPU reference."""
    from epfl_megatron_amd.ops.attention import flash_attn_qkvpacked
    from epfl_megatron_amd.ops.rope import rope_table
    torch.manual_seed(9 + s)
    cos, sin = rope_table(hd, 8192, DEV)
    pos = None
    if with_pos:
        pos = (torch.arange(s)[None, :] + torch.tensor([[3], [700]])[:b]).to(DEV)
    x = torch.randn(s, b, ng * (r + 2) * hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = flash_attn_qkvpacked(x.clone(), ng, r, hd, causal=True, rope=(cos, sin), position_ids=pos)
    xr = x.detach().float().cpu().requires_grad_()
    orf = flash_attn_qkvpacked(xr, ng, r, hd, causal=True, rope=(cos.cpu(), sin.cpu()),
                               position_ids=None if pos is None else pos.cpu())
    _close(o.cpu(), orf, 3e-2, 3e-2, "qkvpacked fwd")
    g = torch.randn_like(o)
    o.backward(g)
    orf.backward(g.float().cpu())
    _close(x.grad.cpu(), xr.grad, 6e-2, 6e-2, "qkvpacked bwd")


def _packed_tokens(b, s, seed, eod=0):
    """Token rows of packed documents: EODs at random places, including
    adjacent EODs (1-token documents), one near the start and a long tail."""
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(1, 100, (b, s), generator=g)
    for i in range(b):
        n = int(torch.randint(1, 9, (1,), generator=g))
        pos = torch.randint(0, s, (n,), generator=g)
        t[i, pos] = eod
        if i == 0 and s > 70:
            t[i, 2] = eod
            t[i, 63:65] = eod  # 1-token document straddling a 64-key tile edge
    return t


@pytest.mark.parametrize("s,b,ng,r,hd", [
    (600, 2, 2, 3, 128),    # GQA, 4-wave grid, dK/dV split over query heads
    (1024, 4, 32, 1, 128),  # Llama-2-7B heads at seq 1k: 8-wave grid, dK/dV kernel epilogue
    (333, 3, 1, 8, 64),     # MQA, head_dim 64
])
def test_flash_attention_document_mask(s, b, ng, r, hd):
    """Packed-document (varlen) masking in the flash kernels (--reset_attention_mask):
    fwd and bwd of the training path against the fp32 reference with the
    same document mask, fused RoPE on and position ids reset per document."""
    from epfl_megatron_amd.ops.attention import flash_attn_qkvpacked
    from epfl_megatron_amd.ops.rope import rope_table
    from epfl_megatron_amd.utils.misc import get_ltor_masks_and_position_ids
    tokens = _packed_tokens(b, s, seed=s + b).to(DEV)
    docs, _, pos = get_ltor_masks_and_position_ids(tokens, 0, True, True, False,
                                                    flash_doc_bounds=True)
    assert docs.dtype == torch.int32 and docs.shape == (2, b, s)
    cos, sin = rope_table(hd, 8192, DEV)
    torch.manual_seed(s)
    x = torch.randn(s, b, ng * (r + 2) * hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = flash_attn_qkvpacked(x.clone(), ng, r, hd, causal=True, rope=(cos, sin), position_ids=pos,
                             doc_bounds=docs)
    ref_dev = DEV if s * s * b * ng * r > 2 ** 26 else "cpu"  # big cases: fp32 reference on the GPU
    xr = x.detach().float().to(ref_dev).requires_grad_()
    orf = flash_attn_qkvpacked(xr, ng, r, hd, causal=True,
                               rope=(cos.to(ref_dev), sin.to(ref_dev)),
                               position_ids=pos.to(ref_dev), doc_bounds=docs.to(ref_dev),
                               ) if ref_dev == "cpu" else None
    if orf is None:  # GPU fp32 reference: the math path on cuda tensors
        from epfl_megatron_amd.ops.attention import attention_ref, _split_qkv5
        from epfl_megatron_amd.ops.rope import apply_rope_ref
        q, k, v = _split_qkv5(xr.view(s, b, ng, r + 2, hd))
        q = apply_rope_ref(q, cos, sin, pos)
        k = apply_rope_ref(k, cos, sin, pos)
        orf = attention_ref(q.transpose(0, 1), k.transpose(0, 1), v.transpose(0, 1), True,
                            hd ** -0.5, doc_bounds=docs).transpose(0, 1).reshape(s, b, -1)
    _close(o.float().cpu(), orf.detach().float().cpu(), 3e-2, 3e-2, "doc-masked fwd")
    g = torch.randn_like(o)
    o.backward(g)
    orf.backward(g.float().to(ref_dev))
    _close(x.grad.float().cpu(), xr.grad.float().cpu(), 6e-2, 6e-2, "doc-masked bwd")


@pytest.mark.parametrize("b,sk,nq,nkv,hd", [(2, 1, 8, 8, 128), (2, 77, 8, 2, 128),
                                              (1, 300, 71, 1, 64), (3, 1000, 64, 8, 128),
                                              (1, 4096, 32, 32, 128), (2, 513, 12, 4, 64)])
def test_flash_decode(b, sk, nq, nkv, hd):
    """Single-token decode against a strided [s, b, nkv, hd] KV cache (the
    inference layout): split-key decode kernel vs fp32 reference."""
    from epfl_megatron_amd.ops.attention import flash_attn_func, attention_ref
    torch.manual_seed(sk + nq)
    kmem = torch.randn(sk + 5, b + 1, nkv, hd, device=DEV, dtype=torch.bfloat16)
    vmem = torch.randn(sk + 5, b + 1, nkv, hd, device=DEV, dtype=torch.bfloat16)
    q = torch.randn(1, b, nq, hd, device=DEV, dtype=torch.bfloat16) * 2
    keys, vals = kmem[:sk, 1:b + 1].transpose(0, 1), vmem[:sk, 1:b + 1].transpose(0, 1)
    with torch.no_grad():
        o = flash_attn_func(q.transpose(0, 1), keys, vals, causal=True)
    orf = attention_ref(q.transpose(0, 1).float(), keys.float(), vals.float(), causal=True)
    _close(o, orf, 2e-2, 2e-2, "decode")


@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (5, 12288, 4096), (16, 4096, 11008),
                                   (4, 32000, 4096), (3, 1376, 512), (24, 4096, 4096),
                                   (32, 4096, 11008), (17, 1376, 512)])
def test_skinny_gemm(M, N, K):
    """Decode-batch weight-streaming GEMM vs fp32 reference, and the linear
    layers' no-grad dispatch to it."""
    C = _ext()
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.02
    assert C.skinny_gemm_supported(M, N, K)
    y = C.skinny_gemm(x, w)
    _close(y, x.float() @ w.float().t(), 2e-2, 2e-2, "skinny gemm")
    assert not C.skinny_gemm_supported(33, N, K) and not C.skinny_gemm_supported(M, N, K + 64)
    from epfl_megatron_amd.parallel.tensor.layers import _skinny_linear
    with torch.no_grad():
        y2 = _skinny_linear(x.view(M, 1, K), w, None, False)
    assert y2 is not None and torch.equal(y2.view(M, N), y)
    assert _skinny_linear(x.view(M, 1, K), w, None, False) is None  # grad mode on: autograd path


@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (8, 1024, 512), (16, 4096, 11008), (3, 512, 384),
                                   (32, 4096, 4096), (19, 1024, 512)])
def test_skinny_fused_norm_residual(M, N, K):
    """Decode projection with the RMSNorm prologue and the residual epilogue
    vs the unfused kernels (rmsnorm_fwd -> skinny GEMM -> add, same roundings)."""
    from epfl_megatron_amd.ops.norms import rms_norm
    C = _ext()
    torch.manual_seed(M * 7 + K)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16) * 3
    g = (torch.rand(K, device=DEV) + 0.5).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.02
    res = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        xn = rms_norm(x, g, 1e-5)
        ref = (C.skinny_gemm(xn, w).float() + res.float()).to(torch.bfloat16)
        y = C.skinny_norm_gemm(x, w, g, 1e-5, res)
        y0 = C.skinny_norm_gemm(x, w, None, 0.0, None)
    assert torch.equal(y0, C.skinny_gemm(x, w))
    _close(y, ref, 2e-2, 2e-2, "norm + residual")
    # fp32 oracle of the whole fused op
    xf = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-5) * g.float()
    _close(y, xf @ w.float().t() + res.float(), 5e-2, 2e-2, "fp32 oracle")


@pytest.mark.parametrize("kind,name", [(0, "swiglu"), (1, "geglu")])
@pytest.mark.parametrize("M,F,K", [(1, 11008, 4096), (8, 512, 512), (16, 1376, 4096),
                                   (3, 2816, 4096), (5, 5632, 4096), (32, 1376, 4096),
                                   (24, 512, 512)])
def test_skinny_fused_glu(M, F, K, kind, name):
    """fc1 decode projection with the norm prologue and the GLU epilogue vs
    rmsnorm -> skinny GEMM -> glu kernel.  F = 11008 / 2816 on 256 CUs run
    the last round as half blocks (1376 = 5 x 256 + 96, 352 = 256 + 96);
    5632 (704 = 2 x 256 + 192) keeps full blocks."""
    from epfl_megatron_amd.ops.norms import rms_norm
    from epfl_megatron_amd.ops.activations import glu
    C = _ext()
    torch.manual_seed(F + M)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    g = (torch.rand(K, device=DEV) + 0.5).to(torch.bfloat16)
    w1 = torch.randn(2 * F, K, device=DEV, dtype=torch.bfloat16) * 0.03
    with torch.no_grad():
        ref = glu(C.skinny_gemm(rms_norm(x, g, 1e-6), w1), name)
        y = C.skinny_norm_glu(x, w1, g, 1e-6, kind)
    assert y.shape == (M, F)
    _close(y, ref, 2e-2, 2e-2, "norm + glu")


@pytest.mark.parametrize("ng,r,hd", [(2, 2, 128), (32, 1, 128), (8, 4, 64)])
@pytest.mark.parametrize("graph_slot", [False, True])
def test_skinny_fused_qkv_rope_cache(ng, r, hd, graph_slot):
    """QKV decode projection with norm + RoPE + KV-cache write vs rmsnorm ->
    skinny GEMM -> rope_qkv_inplace -> cache copies; the cache outside the
    written slot is untouched."""
    from epfl_megatron_amd.ops.norms import rms_norm
    from epfl_megatron_amd.ops.rope import rope_table, rope_qkv_inplace
    C = _ext()
    torch.manual_seed(ng * r + hd)
    b, K, L, B, b0, slot = 3, 512, 40, 5, 1, 17
    N = ng * (r + 2) * hd
    x = torch.randn(b, K, device=DEV, dtype=torch.bfloat16)
    g = (torch.rand(K, device=DEV) + 0.5).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    cos, sin = rope_table(hd, 64, DEV)
    pos = torch.tensor([[5], [17], [40]], device=DEV)
    kmem = torch.randn(L, B, ng, hd, device=DEV, dtype=torch.bfloat16)
    vmem = torch.randn(L, B, ng, hd, device=DEV, dtype=torch.bfloat16)
    k0, v0 = kmem.clone(), vmem.clone()
    with torch.no_grad():
        mixed = C.skinny_gemm(rms_norm(x, g, 1e-5), w).view(1, b, ng, r + 2, hd)
        rope_qkv_inplace(mixed, cos, sin, pos)
        q_ref = mixed[0, :, :, :r].reshape(b, -1)
        kc, vc = kmem[:, b0:b0 + b], vmem[:, b0:b0 + b]
        st = torch.tensor([slot], device=DEV) if graph_slot else None
        q = C.skinny_qkv_rope_cache(x, w, g, 1e-5, ng, r, hd, cos, sin, pos, kc, vc, st,
                                    0 if graph_slot else slot)
    _close(q, q_ref, 2e-2, 2e-2, "q")
    _close(kmem[slot, b0:b0 + b], mixed[0, :, :, r], 2e-2, 2e-2, "k slot")
    _close(vmem[slot, b0:b0 + b], mixed[0, :, :, r + 1], 2e-2, 2e-2, "v slot")
    keep = torch.ones(L, B, dtype=torch.bool, device=DEV)
    keep[slot, b0:b0 + b] = False
    assert torch.equal(kmem[keep], k0[keep]) and torch.equal(vmem[keep], v0[keep])


@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (8, 12288, 4096), (16, 4096, 11008),
                                   (3, 1024, 8192), (5, 512, 512), (1, 22016, 4096),
                                   (32, 12288, 4096), (20, 4096, 11008)])
def test_skinny_packed_weights_match_row_major(M, N, K):
    """The decode-packed weight layout (ops/decode_pack.py) feeds every lane
    the same k indices in the same order as the row-major stream: plain,
    norm + residual, norm + GLU and QKV + RoPE + cache outputs are bit-equal
    across the persistent (K = 4096 / 8192) and per-block (K = 11008 / 512)
    forms; N = 22016 is Llama-2-7B's fc1, whose last round runs as half units
    (1376 blocks = 5 x 256 + 96 on 256 CUs) from the packed half-unit tail."""
    from epfl_megatron_amd.ops import decode_pack
    from epfl_megatron_amd.ops.rope import rope_table
    C = _ext()
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    g = (torch.rand(K, device=DEV) + 0.5).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.02
    res = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    wp = decode_pack.pack(w)
    assert torch.equal(decode_pack.unpack(wp), w)
    with torch.no_grad():
        assert torch.equal(C.skinny_gemm(x, wp, True), C.skinny_gemm(x, w))
        assert torch.equal(C.skinny_norm_gemm(x, wp, g, 1e-5, res, True),
                           C.skinny_norm_gemm(x, w, g, 1e-5, res))
        tail = C.skinny_glu_half_tail(N // 2, K, True, M)
        wg = decode_pack.pack(w, glu=True, half_tail=tail)
        assert torch.equal(decode_pack.unpack(wg, glu=True, half_tail=tail), w)
        for kind in (0, 1):
            assert torch.equal(C.skinny_norm_glu(x, wg, g, 1e-6, kind, True, tail),
                               C.skinny_norm_glu(x, w, g, 1e-6, kind)), kind
        hd = 128
        if N % (3 * hd) == 0:
            ng = N // (3 * hd)
            cos, sin = rope_table(hd, 64, DEV)
            pos = torch.arange(M, device=DEV).view(M, 1) + 3
            caches = [torch.zeros(8, M, ng, hd, device=DEV, dtype=torch.bfloat16) for _ in range(4)]
            qa = C.skinny_qkv_rope_cache(x, wp, g, 1e-5, ng, 1, hd, cos, sin, pos, caches[0],
                                         caches[1], None, 2, True)
            qb = C.skinny_qkv_rope_cache(x, w, g, 1e-5, ng, 1, hd, cos, sin, pos, caches[2],
                                         caches[3], None, 2)
            assert torch.equal(qa, qb) and torch.equal(caches[0], caches[2])
            assert torch.equal(caches[1], caches[3])
    # the cached copy follows in-place updates of the parameter
    p1 = decode_pack.packed(w)
    assert p1 is decode_pack.packed(w)
    w.mul_(2)
    assert torch.equal(decode_pack.packed(w), decode_pack.pack(w))


def test_flash_attention_kvcache_causal_offset():
    """sq < sk (decode with cache): bottom-right aligned causal mask."""
    from epfl_megatron_amd.ops.attention import flash_attn_func, attention_ref
    torch.manual_seed(10)
    q = torch.randn(2, 5, 8, 128, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(2, 70, 2, 128, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(2, 70, 2, 128, device=DEV, dtype=torch.bfloat16)
    o = flash_attn_func(q, k, v, causal=True)
    orf = attention_ref(q.float(), k.float(), v.float(), causal=True)
    _close(o, orf, 2e-2, 2e-2, "kv-cache attention")


@pytest.mark.parametrize("M,N,K", [(32, 256, 256), (96, 512, 256), (1024, 768, 512),
                                   (8192, 256, 512), (16384, 1536, 512), (16544, 1280, 1024),
                                   (16384, 4352, 4096),
                                   # ragged last tiles: Llama-2-7B FFN shards at TP=8
                                   (4096, 2752, 4096), (4096, 4096, 1376), (2048, 264, 520)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_wgrad_gemm(M, N, K, dtype):
    """Hand-written MFMA wgrad (csrc/gemm_wgrad.hip) vs fp32 reference, beta 1 and 0."""
    C = _ext()
    torch.manual_seed(0)
    dy = torch.randn(M, N, device=DEV, dtype=dtype)
    x = torch.randn(M, K, device=DEV, dtype=dtype)
    g = torch.randn(N, K, device=DEV, dtype=torch.float32)
    ref = g + dy.float().t() @ x.float()
    assert C.wgrad_supported(M, N, K)
    C.wgrad_gemm(dy, x, g, True)
    _close(g, ref, atol=1e-3 * math.sqrt(M), msg="accumulate")
    g2 = torch.full((N, K), float("nan"), device=DEV)
    C.wgrad_gemm(dy, x, g2, False)
    _close(g2, dy.float().t() @ x.float(), atol=1e-3 * math.sqrt(M), msg="store")
    assert not C.wgrad_supported(M, N + 4, K)
    assert not C.wgrad_supported(M + 16, N, K)


@pytest.mark.parametrize("variant", [4, 8])
@pytest.mark.parametrize("M,N,K", [(128, 256, 256), (1024, 768, 512), (2048, 264, 520),
                                   (4096, 4096, 1376), (16384, 4096, 4096), (8192, 8448, 2048)])
def test_wgrad_gemm_variants(variant, M, N, K):
    """The persistent 4-wave kernel (default) and the 8-wave ping-pong kernel on
    the same data: ragged edges, several tiles per workgroup, partial rounds."""
    C = _ext()
    torch.manual_seed(3)
    dy = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    g0 = torch.randn(N, K, device=DEV, dtype=torch.float32)
    C.wgrad_set_variant(variant)
    try:
        g = g0.clone()
        C.wgrad_gemm(dy, x, g, True)
        g2 = torch.full((N, K), float("nan"), device=DEV)
        C.wgrad_gemm(dy, x, g2, False)
        g3 = torch.full((N, K), float("nan"), device=DEV)
        C.wgrad_gemm(dy, x, g3, False)
    finally:
        C.wgrad_set_variant(4)  # the default
    ref = dy.float().t() @ x.float()
    _close(g, g0 + ref, atol=1e-3 * math.sqrt(M), msg="accumulate")
    _close(g2, ref, atol=1e-3 * math.sqrt(M), msg="store")
    assert torch.equal(g2, g3)  # deterministic


@pytest.mark.parametrize("world,c,R,N,K", [
    (8, 2, 256, 1536, 4096),   # 7B TP8 qkv shard, piece-major SP gather (split-K tail path)
    (8, 2, 256, 4096, 1376),   # row-parallel fc2 shard: natural X read piece-major
    (4, 4, 64, 512, 768),      # more pieces than 2, small groups
    (2, 2, 4096, 4096, 4096),  # whole-tile rounds (no split)
])
def test_wgrad_gemm_token_map(world, c, R, N, K):
    """x_map: X's rows are a two-level permutation of dY's tokens (the SP
    pipeline's piece-major gathers vs natural rows), read by the kernel
    without a permutation copy; == the fp32 reference on the permuted X,
    bitwise equal to the kernel on an explicitly permuted copy, and close to
    the 8-wave kernel's token-map path (the 4-wave kernel runs the whole-tile
    rounds and the split tails of these shapes)."""
    from epfl_megatron_amd.parallel.tensor.layers import _apply_token_map
    C = _ext()
    torch.manual_seed(4)
    M = world * c * R
    dy = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    for xm in ([R, c, world * R, R], [R, world, c * R, R]):
        xp = _apply_token_map(x, tuple(xm), M)
        g = torch.zeros(N, K, device=DEV)
        C.wgrad_gemm(dy, x, g, False, xm)
        g_ref = torch.zeros(N, K, device=DEV)
        C.wgrad_gemm(dy, xp.contiguous(), g_ref, False)
        assert torch.equal(g, g_ref), xm
        _close(g, dy.float().t() @ xp.float(), atol=1e-3 * math.sqrt(M), msg=f"map {xm}")
        C.wgrad_set_variant(8)  # the 8-wave kernel's token-map path on the same data
        try:
            g8 = torch.zeros(N, K, device=DEV)
            C.wgrad_gemm(dy, x, g8, False, xm)
        finally:
            C.wgrad_set_variant(4)
        _close(g8, g, atol=1e-3 * math.sqrt(M), msg=f"8-wave map {xm}")
    with pytest.raises(RuntimeError):
        C.wgrad_gemm(dy, x, torch.zeros(N, K, device=DEV), False, [R + 16, c, world * R, R])


def test_wgrad_plan():
    """Split-K planning (cost model): small grids split every tile, a partial
    last round splits only its tiles (7B fc1: 1376 tiles = 5 rounds + 96)."""
    C = _ext()
    assert list(C.wgrad_plan(16384, 22016, 4096)) == [1280, 1280, 96, 2]
    assert list(C.wgrad_plan(16384, 12288, 4096)) == [768, 768, 0, 1]  # 3 full rounds
    assert list(C.wgrad_plan(16384, 4352, 4096)) == [256, 256, 16, 8]
    assert list(C.wgrad_plan(16384, 1536, 512)) == [0, 0, 12, 8]
    assert list(C.wgrad_plan(1024, 768, 512)) == [6, 6, 0, 1]  # too few tokens to split
    # ragged 11 x 16 tiles: 2 x 176 pieces would take two rounds -> unsplit
    assert list(C.wgrad_plan(16384, 2752, 4096)) == [176, 176, 0, 1]
    assert list(C.wgrad_plan(16384, 1536, 4096)) == [0, 0, 96, 2]  # 2 x 96 in one round
    # 7B TP8 dense shard: 8 pieces of whole 64-token steps (the 4-wave kernel's
    # split form), not 7 (the cheapest split wins, not the first clear win)
    assert list(C.wgrad_plan(16384, 4096, 512)) == [0, 0, 32, 8]


def test_lt_gemm_layouts():
    """hipBLASLt wrapper with explicit solution selection: all three training layouts."""
    C = _ext()
    torch.manual_seed(1)
    M, N, K = 256, 384, 512
    X = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    W = torch.randn(N, K, device=DEV, dtype=torch.bfloat16)
    dY = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    Y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    algos = C.lt_algos(X, False, W, True, Y, 0.0, 4)
    assert algos
    C.lt_gemm(X, False, W, True, Y, 1.0, 0.0, algos[-1])
    _close(Y, X.float() @ W.float().t(), atol=0.5, rtol=2e-2, msg="fwd")
    G = torch.randn(N, K, device=DEV)
    G0 = G.clone()
    C.lt_gemm(dY, True, X, False, G, 1.0, 1.0, -1)
    _close(G, G0 + dY.float().t() @ X.float(), atol=0.05, rtol=1e-3, msg="wgrad")


def test_linear_wgrad_fresh_and_accumulate():
    """_LinearFn wgrad path: fresh main_grad stores, later micro-batches accumulate."""
    from epfl_megatron_amd.parallel.tensor.layers import _wgrad_into_main_grad
    torch.manual_seed(2)
    w = torch.nn.Parameter(torch.randn(512, 256, device=DEV, dtype=torch.bfloat16))
    w.main_grad = torch.full((512, 256), 7.0, device=DEV)
    w._mg_fresh = True
    ref = torch.zeros(512, 256, device=DEV)
    for _ in range(3):
        dy = torch.randn(128, 512, device=DEV, dtype=torch.bfloat16)
        x = torch.randn(128, 256, device=DEV, dtype=torch.bfloat16)
        _wgrad_into_main_grad(w, dy, x)
        ref += dy.float().t() @ x.float()
    _close(w.main_grad, ref, atol=0.05, msg="main_grad")


@pytest.mark.parametrize("R,C", [(64, 64), (128, 320), (4096, 704)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_transpose16(R, C, dtype):
    """csrc/transpose.hip: exact transpose (bit copy), shape gate."""
    C_ = _ext()
    torch.manual_seed(5)
    x = torch.randn(R, C, device=DEV, dtype=dtype)
    y = torch.full((C, R), float("nan"), device=DEV, dtype=dtype)
    C_.transpose16(x, y)
    assert torch.equal(y, x.t())
    assert C_.transpose16_supported(R, C) and not C_.transpose16_supported(R + 32, C)


def test_linear_tn_layouts(monkeypatch):
    """dgrad through the cached W^T equals the plain product; a new
    training-step generation picks up an updated weight."""
    from epfl_megatron_amd.parallel.tensor import layers as L
    monkeypatch.setattr(L, "_DGRAD_WT", True)
    torch.manual_seed(4)
    w = torch.nn.Parameter(torch.randn(384, 256, device=DEV, dtype=torch.bfloat16) * 0.05)
    w.main_grad = torch.zeros(384, 256, device=DEV)
    x = torch.randn(128, 256, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    for step in range(2):
        L.new_weight_transpose_generation()
        w._mg_fresh = True
        x.grad = None
        y = L.linear_with_grad_accumulation_and_async_allreduce(x, w, None, True, False, False)
        g = torch.randn_like(y)
        y.backward(g)
        assert w._wt_cache[1].shape == (256, 384)
        _close(x.grad, g.float() @ w.detach().float(), atol=0.05, rtol=2e-2, msg=f"dgrad {step}")
        _close(w.main_grad, g.float().t() @ x.detach().float(), atol=0.05, rtol=1e-2,
               msg=f"wgrad {step}")
        with torch.no_grad():
            w.data.mul_(-0.5)  # an optimizer-style update that bypasses the version counter


def test_flash_attention_bwd_kv_longer():
    """Backward with sk > sq (bottom-right causal alignment) and ragged tiles."""
    from epfl_megatron_amd.ops.attention import flash_attn_func, attention_ref
    torch.manual_seed(11)
    q = torch.randn(1, 100, 4, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(1, 230, 2, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(1, 230, 2, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = flash_attn_func(q, k, v, causal=True)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = attention_ref(qr, kr, vr, causal=True)
    g = torch.randn_like(o)
    o.backward(g)
    orf.backward(g.float())
    _close(q.grad, qr.grad, 5e-2, 5e-2, "dq (sk > sq)")
    _close(k.grad, kr.grad, 5e-2, 5e-2, "dk (sk > sq)")
    _close(v.grad, vr.grad, 5e-2, 5e-2, "dv (sk > sq)")


# ------------------------------------------------------ fused bias-dropout-add
def test_bias_dropout_add_mask_bit_exact():
    """GPU mask == the NumPy Philox-4x32-10 transcription (known-answer checked
    on CPU), output == residual + where(mask, (x + x2 + bias) / (1 - p), 0)."""
    from epfl_megatron_amd.ops._ext import ext
    from epfl_megatron_amd.ops.dropout import philox_keep_mask
    torch.manual_seed(3)
    s, b, h, p = 37, 3, 256, 0.3
    x, x2, r = (torch.randn(s, b, h, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    bias = torch.randn(h, device=DEV, dtype=torch.bfloat16)
    seed, offset = 0x1234ABCD5678, 4096
    out = ext().bias_dropout_add_fwd(x, x2, bias, r, p, seed, offset)
    keep = torch.from_numpy(philox_keep_mask(x.numel(), p, seed, offset)).view(s, b, h).to(DEV)
    ref = r.float() + torch.where(keep, (x.float() + x2.float() + bias.float()) / (1 - p),
                                  torch.zeros((), device=DEV))
    _close(out, ref, 2e-2, 2e-2, "bias_dropout_add fwd")
    assert abs(keep.float().mean().item() - (1 - p)) < 0.01
    dout = torch.randn_like(x)
    dx = ext().bias_dropout_add_bwd(dout, p, seed, offset)
    _close(dx, torch.where(keep, dout.float() / (1 - p), torch.zeros((), device=DEV)), 1e-2,
           1e-2, "bias_dropout_add bwd")


def test_bias_dropout_add_autograd_and_rng_stream():
    """Through the op: grads (dx = dx2 = mask*dout/(1-p), dbias = sum, dres = dout);
    consecutive calls draw fresh masks; re-seeding reproduces them; the TP RNG
    tracker's fork gives a different stream (sequence-parallel dropout)."""
    from epfl_megatron_amd.ops.dropout import bias_dropout_add
    from epfl_megatron_amd.parallel.tensor.random import get_cuda_rng_tracker
    torch.manual_seed(4)
    x = torch.randn(64, 2, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn_like(x, requires_grad=True)
    bias = torch.randn(128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    torch.cuda.manual_seed(11)
    y1 = bias_dropout_add(x, bias, r, 0.25, True)
    y2 = bias_dropout_add(x, bias, r, 0.25, True)
    assert not torch.equal(y1, y2)
    torch.cuda.manual_seed(11)
    assert torch.equal(bias_dropout_add(x, bias, r, 0.25, True), y1)
    g = torch.randn_like(y1)
    y1.backward(g)
    from epfl_megatron_amd.ops.dropout import philox_keep_mask
    keep = torch.from_numpy(philox_keep_mask(x.numel(), 0.25, 11, 0)).view_as(x).to(DEV)
    dx = torch.where(keep, g.float() / 0.75, torch.zeros((), device=DEV))
    _close(x.grad, dx, 2e-2, 2e-2, "dx")
    _close(r.grad, g.float(), 0, 0, "dres")
    _close(bias.grad, dx.view(-1, 128).sum(0), 5e-2, 5e-2, "dbias")
    tracker = get_cuda_rng_tracker()
    tracker.reset()
    tracker.add("model-parallel-rng", 999)
    torch.cuda.manual_seed(11)
    with tracker.fork():
        y3 = bias_dropout_add(x, bias, r, 0.25, True)
    assert not torch.equal(y3, y1)


def test_deterministic_attention_backward_and_wgrad():
    """Deterministic mode by construction: the FA backward has no
    atomics (dK/dV summed over a GQA group inside one workgroup, dQ by the
    query-owning workgroup) and the wgrad GEMM reduces each tile in one
    workgroup, so repeated runs are bitwise identical."""
    from epfl_megatron_amd.ops.attention import flash_attn_func
    torch.manual_seed(5)
    q = torch.randn(2, 512, 8, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(2, 512, 2, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(2, 512, 2, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(2, 512, 8, 128, device=DEV, dtype=torch.bfloat16)
    outs = []
    for _ in range(3):
        q.grad = k.grad = v.grad = None
        flash_attn_func(q, k, v, causal=True).backward(g)
        outs.append((q.grad.clone(), k.grad.clone(), v.grad.clone()))
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)
    C = _ext()
    dy = torch.randn(4096, 512, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(4096, 768, device=DEV, dtype=torch.bfloat16)
    g0 = torch.randn(512, 768, device=DEV)
    res = []
    for _ in range(3):
        gg = g0.clone()
        C.wgrad_gemm(dy, x, gg, True)
        res.append(gg)
    assert torch.equal(res[0], res[1]) and torch.equal(res[0], res[2])


@pytest.mark.parametrize("W,causal,nq,nkv,hd,zigzag", [
    (4, True, 8, 2, 128, False), (2, False, 4, 4, 64, False), (3, True, 6, 1, 128, False),
    (4, True, 8, 2, 128, True), (2, True, 4, 4, 64, True)])
def test_ring_attention_kernels(W, causal, nq, nkv, hd, zigzag):
    """Context-parallel ring attention (parallel/context.py) with the HIP
    FlashAttention kernels per (local Q, K/V chunk) pair: LSE merge in the
    forward, global-LSE pair backward; W ranks simulated in one process."""
    from epfl_megatron_amd.ops.attention import attention_ref
    from epfl_megatron_amd.parallel.context import ring_attention_simulated
    torch.manual_seed(W * 10 + hd)
    b, c = 2, 192
    s = W * c
    q = torch.randn(b, s, nq, hd, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(b, s, nkv, hd, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(b, s, nkv, hd, device=DEV, dtype=torch.bfloat16)
    go = torch.randn(b, s, nq, hd, device=DEV, dtype=torch.bfloat16)
    from epfl_megatron_amd.parallel.context import zigzag_slice
    share = (lambda t, i: zigzag_slice(t, 1, i, W)) if zigzag else \
        (lambda t, i: t[:, i * c:(i + 1) * c])  # noqa: E731
    ch = lambda t: [share(t, i).contiguous() for i in range(W)]  # noqa: E731
    outs, (dqs, dks, dvs) = ring_attention_simulated(ch(q), ch(k), ch(v), causal, grad_outs=ch(go),
                                                     zigzag=zigzag)
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    ref = attention_ref(qr, kr, vr, causal=causal)
    ref.backward(go.float())
    for got, want, tol, name in ((outs, ref.detach(), 2e-2, "fwd"), (dqs, qr.grad, 6e-2, "dq"),
                                 (dks, kr.grad, 6e-2, "dk"), (dvs, vr.grad, 6e-2, "dv")):
        _close(torch.cat(got, 1), torch.cat([share(want, i) for i in range(W)], 1), tol, tol,
               f"ring {name}")


@pytest.mark.parametrize("W,nq,nkv,hd,zigzag", [(4, 8, 2, 128, True), (2, 4, 4, 64, False),
                                                  (3, 6, 1, 128, True)])
def test_ring_attention_kernels_document_masks(W, nq, nkv, hd, zigzag):
    """Context parallelism with packed documents (--reset_attention_mask): the
    pair kernels take per-pair local document arrays, off-diagonal pairs run
    the causal kernel with offset sk (document starts only) and split into
    square quarters; vs the fp32 full-sequence document-masked reference.
    Some rows of an off-diagonal pair see no key (their document starts after
    the K chunk): LSE -inf, merged away."""
    from epfl_megatron_amd.ops.attention import attention_ref
    from epfl_megatron_amd.parallel.context import ring_attention_simulated, zigzag_slice
    from epfl_megatron_amd.utils.misc import doc_bounds
    torch.manual_seed(W * 100 + hd)
    b, c = 2, 192
    s = W * c
    tok = torch.randint(1, 100, (b, s))
    for i in range(b):
        tok[i, torch.randperm(s - 1)[:3 + 2 * i]] = 0
    docs = doc_bounds(tok, 0).to(DEV)
    q = torch.randn(b, s, nq, hd, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(b, s, nkv, hd, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(b, s, nkv, hd, device=DEV, dtype=torch.bfloat16)
    go = torch.randn(b, s, nq, hd, device=DEV, dtype=torch.bfloat16)
    share = (lambda t, i: zigzag_slice(t, 1, i, W)) if zigzag else \
        (lambda t, i: t[:, i * c:(i + 1) * c])  # noqa: E731
    ch = lambda t: [share(t, i).contiguous() for i in range(W)]  # noqa: E731
    outs, (dqs, dks, dvs) = ring_attention_simulated(ch(q), ch(k), ch(v), True, grad_outs=ch(go),
                                                     zigzag=zigzag, docs=docs)
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    ref = attention_ref(qr, kr, vr, causal=True, doc_bounds=docs)
    ref.backward(go.float())
    for got, want, tol, name in ((outs, ref.detach(), 2e-2, "fwd"), (dqs, qr.grad, 6e-2, "dq"),
                                 (dks, kr.grad, 6e-2, "dk"), (dvs, vr.grad, 6e-2, "dv")):
        _close(torch.cat(got, 1), torch.cat([share(want, i) for i in range(W)], 1), tol, tol,
               f"ring docs {name}")


@pytest.mark.gpu
def test_ring_pair_kernels_on_sequence_major_views():
    """The model's context-parallel path hands the ring [s, b, n, d] tensors
    transposed to [b, s, n, d] (models/transformer.py
    _context_parallel_forward): the pair kernels read them through strides and
    must match the contiguous layout bit for bit."""
    from epfl_megatron_amd.parallel.context import _pair_bwd, _pair_fwd
    torch.manual_seed(7)
    s, b, nq, nkv, hd = 320, 2, 8, 2, 128
    q = torch.randn(s, b, nq, hd, device=DEV, dtype=torch.bfloat16).transpose(0, 1)
    k = torch.randn(s, b, nkv, hd, device=DEV, dtype=torch.bfloat16).transpose(0, 1)
    v = torch.randn(s, b, nkv, hd, device=DEV, dtype=torch.bfloat16).transpose(0, 1)
    do = torch.randn(s, b, nq, hd, device=DEV, dtype=torch.bfloat16).transpose(0, 1)
    for causal in (True, False):
        o1, l1 = _pair_fwd(q, k, v, causal, hd ** -0.5)
        o2, l2 = _pair_fwd(q.contiguous(), k.contiguous(), v.contiguous(), causal, hd ** -0.5)
        assert torch.equal(o1, o2) and torch.equal(l1, l2)
        g1 = _pair_bwd(q, k, v, o1, l1, do, causal, hd ** -0.5)
        g2 = _pair_bwd(q.contiguous(), k.contiguous(), v.contiguous(), o2, l2, do.contiguous(),
                       causal, hd ** -0.5)
        for a, c in zip(g1, g2):
            assert torch.equal(a, c)


def test_rope_qkv_autograd_matches_reference():
    """ops/rope.py rope_qkv (the context-parallel path's RoPE: HIP kernel
    forward, inverse rotation in the backward) vs apply_rope_ref autograd."""
    from epfl_megatron_amd.ops.rope import apply_rope_ref, rope_qkv, rope_table
    torch.manual_seed(4)
    s, b, g, r, hd = 40, 2, 2, 3, 128
    cos, sin = rope_table(hd, 256, DEV)
    pos = torch.randint(0, 256, (b, s), device=DEV)
    x = torch.randn(s, b, g, r + 2, hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = rope_qkv(x, cos, sin, pos)
    gy = torch.randn_like(y)
    y.backward(gy)
    xr = x.detach().float().requires_grad_()
    qk = apply_rope_ref(xr[:, :, :, :r + 1].reshape(s, b, g * (r + 1), hd), cos, sin, pos)
    yr = torch.cat([qk.view(s, b, g, r + 1, hd), xr[:, :, :, r + 1:]], 3)
    yr.backward(gy.float())
    _close(y, yr, 2e-2, 1e-2, "rope_qkv fwd")
    _close(x.grad, xr.grad, 2e-2, 1e-2, "rope_qkv bwd")


@pytest.mark.parametrize("b,V,dtype", [(1, 32000, torch.bfloat16), (5, 1003, torch.bfloat16),
                                       (3, 32000, torch.float32), (16, 4096, torch.float16)])
def test_greedy_tail_matches_torch(b, V, dtype):
    """csrc/decode_tail.hip: per-row argmax (first maximum, as torch.argmax),
    token / history writes, position increment, and the step / slot / key-count
    increments by the last workgroup; twice, so the arrival counter re-arms."""
    C = _ext()
    torch.manual_seed(b * V)
    full = torch.randn(b, (V + 5 + 7) // 8 * 8, device=DEV).to(dtype)
    logits = full[:, :V]  # a strided view, rows 16-B aligned
    logits[:, V // 3] = logits.max(1).values  # ties: the first index wins
    tokens = torch.zeros(b, dtype=torch.long, device=DEV)
    history = torch.full((b, 8), -1, dtype=torch.long, device=DEV)
    step = torch.tensor([2], dtype=torch.long, device=DEV)
    pos = torch.arange(b, dtype=torch.long, device=DEV) + 10
    slot = torch.tensor([40], dtype=torch.long, device=DEV)
    kvl = torch.tensor([41], dtype=torch.int32, device=DEV)
    counter = torch.zeros(1, dtype=torch.int32, device=DEV)
    for it in range(2):
        C.greedy_tail(logits, tokens, history, step, pos, slot, kvl, counter)
        want = logits.float().argmax(1)
        assert torch.equal(tokens, want)
        assert torch.equal(history[:, 2 + it], want)
    assert torch.all(history[:, :2] == -1) and torch.all(history[:, 4:] == -1)
    assert step.item() == 4 and slot.item() == 42 and kvl.item() == 43 and counter.item() == 0
    assert torch.equal(pos, torch.arange(b, device=DEV) + 12)

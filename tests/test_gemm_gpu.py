"""Numerics of the hand-written NT GEMM (csrc/gemm_nt.hip) and its fused GLU
epilogues against plain PyTorch fp32 references.

Forward  Y = X W^T, dgrad dX = dY (W^T)^T, fc1 forward with the GLU fused
(pre-activation + y = x1 * act(x2)) and fc2 dgrad with the GLU backward fused
(reference MLP: megatron/model/transformer.py:92-123, GLU order
megatron/model/glu_activations.py:18-21).  Shapes cover the Llama-2-7B,
70B-TP8-rank and Falcon projections plus ragged M / N tails.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ext():
    from epfl_megatron_amd.ops._ext import ext
    return ext()


def _rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _rand(*shape, dtype=torch.bfloat16, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(dtype)


@pytest.mark.parametrize("M,N,K", [
    (256, 256, 32),        # one tile, one subtile
    (512, 768, 64),        # two subtiles (short ring)
    (300, 264, 96),        # ragged M and N, three subtiles
    (1000, 1000, 4096),    # ragged, long K
    (2048, 4096, 4096),    # 7B o-proj shape class
    (1024, 1536, 8192),    # 70B TP8 qkv rank shape (N = 1536)
    (777, 2752, 1024),     # 70B TP8 fc1 rank width (2752 = 10.75 tiles)
    (512, 9216, 8192),     # Falcon-40B TP4 qkv width
])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gemm_nt(M, N, K, dtype):
    torch.manual_seed(0)
    a = _rand(M, K, dtype=dtype)
    b = _rand(N, K, dtype=dtype, scale=K ** -0.5)
    c = _ext().gemm_nt(a, b)
    ref = a.float() @ b.float().t()
    assert c.dtype == dtype and c.shape == (M, N)
    assert _rel_err(c, ref) < 8e-3
    # the rounding of each element is one rounding of an fp32 sum
    tol = (2 ** -7 if dtype == torch.bfloat16 else 2 ** -10) * ref.abs() + 2e-2
    assert ((c.float() - ref).abs() <= tol).all()


@pytest.mark.parametrize("variant", [4, 6, 8])
@pytest.mark.parametrize("M,N,K", [
    (256, 256, 128),       # one tile, two K-steps (the persistent kernel's minimum)
    (300, 264, 192),       # ragged M and N, odd number of K-steps
    (1000, 1000, 4096),    # ragged, long K, several tiles per workgroup
    (4096, 4096, 1024),    # 256 tiles: one round
    (8448, 4096, 640),     # 528 tiles: a partial last round, odd K-steps per tile
])
def test_gemm_nt_variants(variant, M, N, K):
    """Every kernel variant (4-wave, persistent, 8-wave) on the same data."""
    torch.manual_seed(1)
    a = _rand(M, K)
    b = _rand(N, K, scale=K ** -0.5)
    C = _ext()
    C.gemm_nt_set_variant(variant)
    try:
        c = C.gemm_nt(a, b)
        c2 = C.gemm_nt(a, b)
    finally:
        C.gemm_nt_set_variant(0)
    ref = a.float() @ b.float().t()
    tol = 2 ** -7 * ref.abs() + 2e-2
    assert ((c.float() - ref).abs() <= tol).all()
    assert torch.equal(c, c2)


def test_gemm_nt_identity_asymmetric():
    """A = I with an asymmetric B exposes any row/col swap of the C-write."""
    n = 256
    a = torch.eye(n, device=DEV, dtype=torch.bfloat16)
    b = (torch.arange(n, device=DEV).view(n, 1) * 3 + torch.arange(n, device=DEV).view(1, n) % 7)
    b = (b % 61).to(torch.bfloat16)
    c = _ext().gemm_nt(a, b)
    assert torch.equal(c.float(), b.float().t())


def test_gemm_nt_strided_out_and_inputs():
    torch.manual_seed(1)
    big = _rand(512, 640)
    a = big[:, 64:576]               # row stride 640, 16-B aligned start
    b = _rand(384, 512, scale=512 ** -0.5)
    out = torch.zeros(512, 400, device=DEV, dtype=torch.bfloat16)
    _ext().gemm_nt(a, b, out[:, :384])
    ref = a.float() @ b.float().t()
    assert _rel_err(out[:, :384], ref) < 8e-3
    assert (out[:, 384:] == 0).all()


def _glu_ref(pre, kind):
    from epfl_megatron_amd.ops.activations import glu_ref
    return glu_ref(pre, kind)


@pytest.mark.parametrize("M,F,K", [(256, 128, 64), (300, 200, 96), (1024, 1376, 512),
                                   (512, 11008 // 4, 4096)])
@pytest.mark.parametrize("kind", ["swiglu", "geglu", "reglu", "liglu"])
def test_gemm_nt_glu_forward(M, F, K, kind):
    torch.manual_seed(2)
    kinds = {"swiglu": 0, "geglu": 1, "reglu": 2, "liglu": 3}
    x = _rand(M, K)
    w1 = _rand(2 * F, K, scale=K ** -0.5)
    pre, y = _ext().gemm_nt_glu(x, w1, kinds[kind])
    ref_pre = x.float() @ w1.float().t()
    assert _rel_err(pre, ref_pre) < 8e-3
    # y is exactly the elementwise op applied to the kernel's own rounded pre
    y_ref = _glu_ref(pre.float(), kind)
    assert _rel_err(y, y_ref) < 8e-3
    assert _rel_err(y, _glu_ref(ref_pre, kind)) < 2e-2


@pytest.mark.parametrize("M,F,K", [(256, 128, 64), (300, 200, 96), (1024, 1376, 512),
                                   (512, 11008 // 4, 4096)])
@pytest.mark.parametrize("kind", ["swiglu", "geglu"])
def test_gemm_nt_dglu_backward(M, F, K, kind):
    torch.manual_seed(3)
    kinds = {"swiglu": 0, "geglu": 1, "reglu": 2, "liglu": 3}
    pre = _rand(M, 2 * F)
    dy = _rand(M, K)
    w2 = _rand(K, F, scale=F ** -0.5)            # fc2 weight [out = K, in = F]
    w2t = w2.t().contiguous()                    # [F, K]
    dpre = _ext().gemm_nt_dglu(dy, w2t, pre, kinds[kind])
    # oracle: autograd through fp32 glu of the same pre, upstream dact = dy @ w2
    p32 = pre.float().requires_grad_(True)
    y = _glu_ref(p32, kind)
    dact = dy.float() @ w2.float()
    y.backward(dact)
    assert dpre.shape == (M, 2 * F)
    assert _rel_err(dpre, p32.grad) < 1.5e-2


@pytest.mark.parametrize("M,F,K", [(256, 128, 128), (300, 200, 192), (1024, 1376, 512),
                                   (4096, 2752, 1024)])
@pytest.mark.parametrize("kind", ["swiglu", "reglu"])
def test_gemm_nt_glu_persistent_matches_oneshot(M, F, K, kind):
    """The persistent kernel's register epilogues (variant 6) give the one-shot
    kernel's GLU forward and backward outputs exactly (same rounding points)."""
    torch.manual_seed(5)
    kinds = {"swiglu": 0, "reglu": 2}
    C = _ext()
    x = _rand(M, K)
    w1 = _rand(2 * F, K, scale=K ** -0.5)
    pre = _rand(M, 2 * F)
    dy = _rand(M, K)
    w2t = _rand(F, K, scale=F ** -0.5)
    outs = {}
    for v in (5, 6):
        C.gemm_nt_set_variant(v)
        try:
            outs[v] = (*C.gemm_nt_glu(x, w1, kinds[kind]), C.gemm_nt_dglu(dy, w2t, pre, kinds[kind]))
        finally:
            C.gemm_nt_set_variant(0)
    for a, b in zip(outs[5], outs[6]):
        assert torch.equal(a, b)
    assert _rel_err(outs[6][0], x.float() @ w1.float().t()) < 8e-3


def test_gemm_nt_matches_unfused_path():
    """Fused fc1 + fc2-dgrad == hipBLASLt matmul + the elementwise GLU kernels."""
    from epfl_megatron_amd.ops.activations import glu
    torch.manual_seed(4)
    M, H, F = 1024, 512, 1376
    x = _rand(M, H)
    w1 = _rand(2 * F, H, scale=H ** -0.5)
    w2 = _rand(H, F, scale=F ** -0.5)
    pre, y = _ext().gemm_nt_glu(x, w1, 0)
    pre_u = x @ w1.t()
    assert _rel_err(pre, pre_u) < 8e-3
    assert _rel_err(y, glu(pre_u)) < 1e-2
    dy = _rand(M, H)
    dpre = _ext().gemm_nt_dglu(dy, w2.t().contiguous(), pre, 0)
    dact = dy @ w2
    dpre_u = _ext().glu_bwd(dact, pre, 0)
    assert _rel_err(dpre, dpre_u) < 1e-2


@pytest.mark.parametrize("M,H,F,kind", [
    (512, 256, 352, "swiglu"),     # F = 11 x 32 (W^T built by torch, not transpose16)
    (1000, 512, 1408, "swiglu"),   # ragged M
    (300, 256, 256, "geglu"),
])
def test_fused_glu_mlp_fwd_bwd_vs_fp32(M, H, F, kind):
    """fc1 + GLU + fc2 forward and backward through parallel.tensor.glu_mlp
    (NT GEMM, GLU in the fc1 epilogue, GLU backward in the fc2 dgrad epilogue)
    against the fp32 torch composition."""
    from epfl_megatron_amd.parallel.tensor import glu_mlp
    torch.manual_seed(1)
    x = _rand(M, H).requires_grad_()
    w1 = _rand(2 * F, H, scale=H ** -0.5).requires_grad_()
    w2 = _rand(H, F, scale=F ** -0.5).requires_grad_()
    dout = _rand(M, H)
    out = glu_mlp(x, w1, w2, kind, sequence_parallel=False, tp_async_allreduce=False,
                  gradient_accumulation_fusion=False)
    out.backward(dout)
    xr, w1r, w2r = (t.detach().float().requires_grad_() for t in (x, w1, w2))
    pre = xr @ w1r.t()
    act = torch.nn.functional.silu if kind == "swiglu" else torch.nn.functional.gelu
    ref = (pre[:, :F] * act(pre[:, F:])) @ w2r.t()
    ref.backward(dout.float())
    assert _rel_err(out, ref) < 1e-2
    assert _rel_err(x.grad, xr.grad) < 2e-2
    assert _rel_err(w1.grad, w1r.grad) < 2e-2
    assert _rel_err(w2.grad, w2r.grad) < 2e-2


@pytest.mark.parametrize("tp,c,R,N,K", [
    (8, 2, 1024, 1536, 4096),   # 7B TP8 s4096 mbs4 rank: chunk rows = s/(tp c) * b
    (4, 2, 200, 264, 96),       # ragged group size, ragged N
    (2, 3, 128, 512, 64),
])
def test_gemm_nt_row_maps(tp, c, R, N, K):
    """Row-group remaps of the chunked TP overlap: A rows gathered from (and C
    rows scattered to) groups of R rows at stride c*R, offset j*R."""
    torch.manual_seed(2)
    b = _rand(N, K, scale=K ** -0.5)
    full = _rand(tp * c * R, K)
    for j in range(c):
        out = _ext().gemm_nt(full, b, a_map=[R, c * R, j * R], m=tp * R)
        ref = full.view(tp, c, R, K)[:, j].reshape(tp * R, K).float() @ b.float().t()
        assert out.shape == (tp * R, N) and _rel_err(out, ref) < 1e-2
    g = _rand(tp * R, K)
    dst = torch.zeros(tp * c * R, N, device=DEV, dtype=torch.bfloat16)
    j = c - 1
    _ext().gemm_nt(g, b, dst, c_map=[R, c * R, j * R])
    v = dst.view(tp, c, R, N)
    assert _rel_err(v[:, j].reshape(tp * R, N), g.float() @ b.float().t()) < 1e-2
    assert v[:, :j].abs().sum().item() == 0
    # fused GLU with a C remap into the full pre / y
    F = 256
    w1 = _rand(2 * F, K, scale=K ** -0.5)
    pre = torch.zeros(tp * c * R, 2 * F, device=DEV, dtype=torch.bfloat16)
    y = torch.zeros(tp * c * R, F, device=DEV, dtype=torch.bfloat16)
    _ext().gemm_nt_glu(g, w1, 0, pre, y, [R, c * R, 0])
    p_ref = g.float() @ w1.float().t()
    y_ref = p_ref[:, :F] * torch.nn.functional.silu(p_ref[:, F:])
    assert _rel_err(pre.view(tp, c, R, 2 * F)[:, 0].reshape(tp * R, -1), p_ref) < 1e-2
    assert _rel_err(y.view(tp, c, R, F)[:, 0].reshape(tp * R, -1), y_ref) < 2e-2
    assert y.view(tp, c, R, F)[:, 1:].abs().sum().item() == 0


@pytest.mark.parametrize("tp,c,R,N,K,dtype,splits", [
    (1, 1, 1024, 1280, 8192, torch.bfloat16, 8),   # 20 tiles: K split 8 ways
    (8, 2, 512, 1280, 8192, torch.bfloat16, 2),    # Llama-2-70B TP8 qkv piece (80 tiles: 2 ways)
    (8, 2, 256, 1280, 8192, torch.bfloat16, 4),    # a half-size piece (40 tiles: 4 ways)
    (8, 2, 256, 1000, 8192, torch.bfloat16, 8),    # ragged N (32 tiles: 8 ways)
    (1, 1, 1000, 1280, 8192, torch.bfloat16, 8),   # ragged M (a partial last m-tile)
    (8, 2, 512, 1280, 8192, torch.float16, 2),     # fp16 operands
    (8, 2, 256, 1024, 4096, torch.bfloat16, 8),    # dense-dgrad-like piece through a C map
])
def test_gemm_nt_split_k(tp, c, R, N, K, dtype, splits):
    """Few-tile products on the persistent kernel split K over fp32 partials
    (gemm_nt_split_reduce_k, fixed order): A / C row maps, ragged M and N,
    fp16, the split count the plan picks, and bitwise-reproducible results."""
    torch.manual_seed(6)
    assert _ext().gemm_nt_ksplit(tp * R, N, K) == splits
    b = _rand(N, K, dtype=dtype, scale=K ** -0.5)
    full = _rand(tp * c * R, K, dtype=dtype)
    j = c - 1
    amap = [R, c * R, j * R] if c > 1 else []
    out = _ext().gemm_nt(full, b, a_map=amap, m=tp * R)
    out2 = _ext().gemm_nt(full, b, a_map=amap, m=tp * R)
    ref = full.view(tp, c, R, K)[:, j].reshape(tp * R, K).float() @ b.float().t()
    assert out.shape == (tp * R, N) and out.dtype == dtype and _rel_err(out, ref) < 1e-2
    assert torch.equal(out, out2)
    if c > 1:
        g = _rand(tp * R, K, dtype=dtype)
        dst = torch.zeros(tp * c * R, N, device=DEV, dtype=dtype)
        _ext().gemm_nt(g, b, dst, c_map=[R, c * R, 0])
        v = dst.view(tp, c, R, N)
        assert _rel_err(v[:, 0].reshape(tp * R, N), g.float() @ b.float().t()) < 1e-2
        assert v[:, 1:].abs().sum().item() == 0


def test_gemm_nt_row_map_out_of_range_refused():
    a = _rand(256, 64)
    b = _rand(256, 64)
    with pytest.raises(RuntimeError):
        _ext().gemm_nt(a, b, a_map=[128, 256, 128], m=256)  # rows 128..383 of a 256-row a

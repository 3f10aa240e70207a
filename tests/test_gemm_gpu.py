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

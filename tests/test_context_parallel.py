"""Context-parallel ring attention (``parallel/context.py``) on gloo / CPU:
every rank's output chunk and its dQ / dK / dV chunks equal full-sequence
attention (fp32 reference), causal and not, MHA and GQA, W = 2 and 4."""
import pytest
import torch

from dist_utils import run_dist


def _full(b, s, nq, nkv, d, seed):
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(b, s, nq, d, generator=g)
    k = torch.randn(b, s, nkv, d, generator=g)
    v = torch.randn(b, s, nkv, d, generator=g)
    go = torch.randn(b, s, nq, d, generator=g)
    return q, k, v, go


def _ring_rank(rank, world, causal, nq, nkv):
    import torch.distributed as dist
    from epfl_megatron_amd.parallel.context import ring_attention
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, s, d = 2, 12 * world, 16
    q, k, v, go = _full(b, s, nq, nkv, d, seed=3)
    c = s // world
    sl = slice(rank * c, (rank + 1) * c)
    ql, kl, vl = (t[:, sl].clone().requires_grad_() for t in (q, k, v))
    out = ring_attention(ql, kl, vl, dist.group.WORLD, causal=causal)
    out.backward(go[:, sl])
    return out.detach(), ql.grad, kl.grad, vl.grad


@pytest.mark.parametrize("world,causal,nq,nkv", [(2, True, 4, 4), (4, True, 4, 2),
                                                 (4, False, 4, 4), (2, False, 6, 2)])
def test_ring_attention_matches_full(world, causal, nq, nkv):
    from epfl_megatron_amd.ops.attention import attention_ref
    res = run_dist(_ring_rank, world, causal, nq, nkv)
    b, s, d = 2, 12 * world, 16
    q, k, v, go = _full(b, s, nq, nkv, d, seed=3)
    qr, kr, vr = (t.clone().requires_grad_() for t in (q, k, v))
    ref = attention_ref(qr, kr, vr, causal=causal)
    ref.backward(go)
    c = s // world
    for rank, (o, dq, dk, dv) in enumerate(res):
        sl = slice(rank * c, (rank + 1) * c)
        torch.testing.assert_close(o, ref.detach()[:, sl], atol=2e-5, rtol=2e-5)
        torch.testing.assert_close(dq, qr.grad[:, sl], atol=5e-5, rtol=5e-5)
        torch.testing.assert_close(dk, kr.grad[:, sl], atol=5e-5, rtol=5e-5)
        torch.testing.assert_close(dv, vr.grad[:, sl], atol=5e-5, rtol=5e-5)


def test_ring_attention_simulated_matches_full():
    """The single-process ring (the GPU kernel test's form) on CPU."""
    from epfl_megatron_amd.ops.attention import attention_ref
    from epfl_megatron_amd.parallel.context import ring_attention_simulated
    W, b, s, nq, nkv, d = 3, 1, 24, 4, 2, 16
    q, k, v, go = _full(b, s, nq, nkv, d, seed=5)
    c = s // W
    ch = lambda t: [t[:, i * c:(i + 1) * c] for i in range(W)]  # noqa: E731
    outs, (dqs, dks, dvs) = ring_attention_simulated(ch(q), ch(k), ch(v), True, grad_outs=ch(go))
    qr, kr, vr = (t.clone().requires_grad_() for t in (q, k, v))
    ref = attention_ref(qr, kr, vr, causal=True)
    ref.backward(go)
    torch.testing.assert_close(torch.cat(outs, 1), ref.detach(), atol=2e-5, rtol=2e-5)
    torch.testing.assert_close(torch.cat(dqs, 1), qr.grad, atol=5e-5, rtol=5e-5)
    torch.testing.assert_close(torch.cat(dks, 1), kr.grad, atol=5e-5, rtol=5e-5)
    torch.testing.assert_close(torch.cat(dvs, 1), vr.grad, atol=5e-5, rtol=5e-5)

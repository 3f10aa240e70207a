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


def _share(t, rank, world, zigzag):
    from epfl_megatron_amd.parallel.context import zigzag_slice
    if zigzag:
        return zigzag_slice(t, 1, rank, world)
    c = t.shape[1] // world
    return t[:, rank * c:(rank + 1) * c]


def _ring_rank(rank, world, causal, nq, nkv, zigzag):
    import torch.distributed as dist
    from epfl_megatron_amd.parallel.context import ring_attention
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, s, d = 2, 12 * world, 16
    q, k, v, go = _full(b, s, nq, nkv, d, seed=3)
    ql, kl, vl = (_share(t, rank, world, zigzag).clone().requires_grad_() for t in (q, k, v))
    out = ring_attention(ql, kl, vl, dist.group.WORLD, causal=causal, zigzag=zigzag)
    out.backward(_share(go, rank, world, zigzag))
    return out.detach(), ql.grad, kl.grad, vl.grad


@pytest.mark.parametrize("world,causal,nq,nkv,zigzag", [
    (2, True, 4, 4, False), (4, True, 4, 2, False), (4, False, 4, 4, False),
    (2, False, 6, 2, False), (2, True, 4, 4, True), (4, True, 4, 2, True),
    (3, True, 6, 2, True)])
def test_ring_attention_matches_full(world, causal, nq, nkv, zigzag):
    from epfl_megatron_amd.ops.attention import attention_ref
    res = run_dist(_ring_rank, world, causal, nq, nkv, zigzag)
    b, s, d = 2, 12 * world, 16
    q, k, v, go = _full(b, s, nq, nkv, d, seed=3)
    qr, kr, vr = (t.clone().requires_grad_() for t in (q, k, v))
    ref = attention_ref(qr, kr, vr, causal=causal)
    ref.backward(go)
    for rank, (o, dq, dk, dv) in enumerate(res):
        sh = lambda t: _share(t, rank, world, zigzag)  # noqa: E731
        torch.testing.assert_close(o, sh(ref.detach()), atol=2e-5, rtol=2e-5)
        torch.testing.assert_close(dq, sh(qr.grad), atol=5e-5, rtol=5e-5)
        torch.testing.assert_close(dk, sh(kr.grad), atol=5e-5, rtol=5e-5)
        torch.testing.assert_close(dv, sh(vr.grad), atol=5e-5, rtol=5e-5)


def test_zigzag_plan_balances_causal_work():
    """Every rank of a zig-zag ring does the same attention work (in units of
    a quarter pair) at every W; the contiguous split does not."""
    from epfl_megatron_amd.parallel.context import _plan
    size = {"all": 2, "first": 1, "second": 1}
    for W in (2, 4, 8):
        def work(r, zz):
            tot = 0
            for j in range(W):
                p = _plan(j, r, True, zz)
                if p is not None:
                    tot += size[p[0]] * size[p[1]] // (2 if p[2] else 1)
            return tot
        # quarter-pair units: diagonal (causal) 2, full pair 4, half pair 2
        assert {work(r, True) for r in range(W)} == {2 * W}
        assert work(0, False) == 2 and work(W - 1, False) == 4 * W - 2


@pytest.mark.parametrize("zigzag", [False, True])
def test_ring_attention_simulated_matches_full(zigzag):
    """The single-process ring (the GPU kernel test's form) on CPU."""
    from epfl_megatron_amd.ops.attention import attention_ref
    from epfl_megatron_amd.parallel.context import ring_attention_simulated
    W, b, s, nq, nkv, d = 3, 1, 24, 4, 2, 16
    q, k, v, go = _full(b, s, nq, nkv, d, seed=5)
    ch = lambda t: [_share(t, i, W, zigzag) for i in range(W)]  # noqa: E731
    outs, (dqs, dks, dvs) = ring_attention_simulated(ch(q), ch(k), ch(v), True, grad_outs=ch(go),
                                                     zigzag=zigzag)
    qr, kr, vr = (t.clone().requires_grad_() for t in (q, k, v))
    ref = attention_ref(qr, kr, vr, causal=True)
    ref.backward(go)
    for got, want in ((outs, ref.detach()), (dqs, qr.grad), (dks, kr.grad), (dvs, vr.grad)):
        for i in range(W):
            torch.testing.assert_close(got[i].float(), _share(want, i, W, zigzag),
                                       atol=5e-5, rtol=5e-5)


def _docs(b, s, seed):
    """Packed-document bounds of random token rows with EOD (token 0) at a
    few random positions: documents cross the chunk / piece boundaries."""
    from epfl_megatron_amd.utils.misc import doc_bounds
    g = torch.Generator().manual_seed(seed)
    tok = torch.randint(1, 50, (b, s), generator=g)
    for i in range(b):
        for p in torch.randperm(s - 1, generator=g)[: 2 + i]:
            tok[i, p] = 0
    return doc_bounds(tok, 0)


def _ring_docs_rank(rank, world, nq, nkv, zigzag):
    import torch.distributed as dist
    from epfl_megatron_amd.parallel.context import ring_attention
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, s, d = 2, 12 * world, 16
    q, k, v, go = _full(b, s, nq, nkv, d, seed=7)
    docs = _docs(b, s, seed=11)
    ql, kl, vl = (_share(t, rank, world, zigzag).clone().requires_grad_() for t in (q, k, v))
    out = ring_attention(ql, kl, vl, dist.group.WORLD, causal=True, zigzag=zigzag, docs=docs)
    out.backward(_share(go, rank, world, zigzag))
    return out.detach(), ql.grad, kl.grad, vl.grad


@pytest.mark.parametrize("world,nq,nkv,zigzag", [(2, 4, 4, False), (2, 4, 2, True),
                                                 (4, 4, 2, True), (3, 6, 2, True)])
def test_ring_attention_document_masks(world, nq, nkv, zigzag):
    """--reset_attention_mask under context parallelism: the ring with the
    whole sequence's document bounds equals full-sequence document-masked
    attention (outputs and dQ / dK / dV of every rank's share)."""
    from epfl_megatron_amd.ops.attention import attention_ref
    res = run_dist(_ring_docs_rank, world, nq, nkv, zigzag)
    b, s, d = 2, 12 * world, 16
    q, k, v, go = _full(b, s, nq, nkv, d, seed=7)
    docs = _docs(b, s, seed=11)
    qr, kr, vr = (t.clone().requires_grad_() for t in (q, k, v))
    ref = attention_ref(qr, kr, vr, causal=True, doc_bounds=docs)
    ref.backward(go)
    for rank, (o, dq, dk, dv) in enumerate(res):
        sh = lambda t: _share(t, rank, world, zigzag)  # noqa: E731
        torch.testing.assert_close(o, sh(ref.detach()), atol=2e-5, rtol=2e-5)
        torch.testing.assert_close(dq, sh(qr.grad), atol=5e-5, rtol=5e-5)
        torch.testing.assert_close(dk, sh(kr.grad), atol=5e-5, rtol=5e-5)
        torch.testing.assert_close(dv, sh(vr.grad), atol=5e-5, rtol=5e-5)


def test_ring_document_pair_arrays():
    """Per-pair local document arrays: first local key at / after each query's
    document start, first local query at / after each key's document end."""
    from epfl_megatron_amd.parallel.context import _pair_docs
    docs = torch.tensor([[[0, 0, 0, 3, 3, 3, 3, 7, 7, 7]], [[3, 3, 3, 7, 7, 7, 7, 10, 10, 10]]],
                        dtype=torch.int32)
    pq, pk = torch.tensor([6, 7, 8, 9]), torch.tensor([1, 2, 3, 4])
    pd = _pair_docs(docs, pq, pk)
    # q 6 (doc [3, 7)) -> first key >= 3 is local 2; q 7..9 (doc [7, 10)) -> 4 (none)
    assert pd[0, 0].tolist() == [2, 4, 4, 4]
    # key 1, 2 end at 3 -> first query >= 3 is local 0; keys 3, 4 end at 7 -> local 1
    assert pd[1, 0].tolist() == [0, 0, 1, 1]

"""Context parallelism: ring attention over a sequence-sharded group.

An optional extension ("context-parallel ring attention over
xGMI for >100k tokens"; the reference has no context parallelism).  The
sequence is split contiguously over the ranks of a group: rank r holds
positions [r*s, (r+1)*s) of Q, K and V.  Attention over the whole sequence is
computed with the FlashAttention kernels on (local Q, one K/V chunk) pairs
while the K/V chunks travel around the ring:

forward   step i: chunk j = (r - i) mod W arrives from the previous rank.  For
          causal attention chunks j > r are skipped, j == r runs the causal
          kernel, j < r the full one.  Each step returns (O_j, LSE_j) and the
          running (O, LSE) merge is the log-sum-exp combine
              LSE = log(e^LSE + e^LSE_j),  O = O e^(LSE_old-LSE) + O_j e^(LSE_j-LSE).
          The next chunk's send / receive (one batched p2p per step through
          ``parallel/comm.py``) is posted before the step's kernel, so the
          transfer overlaps the attention.
backward  with the GLOBAL O and LSE every (local Q, chunk j) pair yields its
          exact share of dQ, dK_j, dV_j from the FlashAttention backward
          (delta = rowsum(dO O) and P = exp(S - LSE) only need the global
          values).  dQ stays local; (K_j, V_j, dK_j, dV_j) travel one hop per
          step and after W hops every chunk is back at its owner with its
          complete dK and dV.

The per-pair kernels are the training kernels (``csrc/flash_attn_fwd.hip`` /
``flash_attn_bwd.hip``: native GQA, LSE in natural log); on CPU tensors the
same math runs in fp32 torch (tests, gloo).  ``ring_attention_simulated`` runs
the W ranks of a ring one after another in one process (kernel-level tests on
one GPU).

Training integration (``--context_parallel_size C``): C consecutive DP ranks
form a context-parallel group (``state.get_context_parallel_group``) and read
the same samples; ``get_batch_on_this_cp_rank`` keeps this rank's contiguous
sequence chunk (global position ids included), self-attention runs
``ring_attention`` (``models/transformer.py``), and ``cp_token_mean`` makes the
per-rank loss the exact whole-sequence token mean once DDP averages gradients
over all DP x CP ranks.
"""
import math

import torch
import torch.distributed as dist

from . import comm


# ---------------------------------------------------------------------------
# one (local Q, K/V chunk) pair
# ---------------------------------------------------------------------------
def _strides(t, r):
    sb, ss, sh, sd = t.stride()
    if sd != 1:
        raise AssertionError("head_dim must be contiguous")
    return [sb, ss, r * sh, sh]


def _pair_fwd(q, k, v, causal, scale):
    """(O [b, s, nq, d] fp32-accurate in q.dtype, LSE [b, nq, s] fp32 natural log)."""
    b, sq, nq, d = q.shape
    sk, nkv = k.shape[1], k.shape[2]
    if not q.is_cuda:
        from ..ops.attention import attention_ref
        o, lse = attention_ref(q, k, v, causal, scale, return_lse=True)
        return o.float(), lse.float()
    from ..ops._ext import ext
    r = nq // nkv
    out = torch.empty_like(q)
    lse = torch.empty(b, nq, sq, dtype=torch.float32, device=q.device)
    ext().flash_attn_fwd(q, k, v, out, lse, b, sq, sk, nq, nkv, d, _strides(q, r),
                         _strides(k, 1)[:3], _strides(v, 1)[:3],
                         [out.stride(0), out.stride(1), out.stride(2)], bool(causal),
                         float(scale), None, None, None, None)
    return out.float(), lse


def _pair_bwd(q, k, v, o, lse, do, causal, scale):
    """dQ, dK, dV of one pair given the GLOBAL output ``o`` and ``lse``."""
    b, sq, nq, d = q.shape
    sk, nkv = k.shape[1], k.shape[2]
    r = nq // nkv
    if not q.is_cuda:
        qf, kf, vf, of, dof = (t.float() for t in (q, k, v, o, do))
        kx = kf.repeat_interleave(r, dim=2)
        vx = vf.repeat_interleave(r, dim=2)
        s = torch.einsum("bqhd,bkhd->bhqk", qf, kx) * scale
        if causal:
            i = torch.arange(sq)[:, None]
            j = torch.arange(sk)[None, :]
            s = s.masked_fill(j > i + (sk - sq), float("-inf"))
        p = torch.exp(s - lse[..., None])
        dv = torch.einsum("bhqk,bqhd->bkhd", p, dof)
        dp = torch.einsum("bqhd,bkhd->bhqk", dof, vx)
        delta = (dof * of).sum(-1).permute(0, 2, 1)[..., None]  # [b, h, q, 1]
        ds = p * (dp - delta)
        dq = torch.einsum("bhqk,bkhd->bqhd", ds, kx) * scale
        dk = torch.einsum("bhqk,bqhd->bkhd", ds, qf) * scale
        dk = dk.view(b, sk, nkv, r, d).sum(3)
        dv = dv.view(b, sk, nkv, r, d).sum(3)
        return dq, dk, dv
    from ..ops._ext import ext
    q, k, v, do = q.contiguous(), k.contiguous(), v.contiguous(), do.contiguous()
    o = o.to(q.dtype).contiguous()
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    ext().flash_attn_bwd(do, q, k, v, o, lse.contiguous(), dq, dk, dv, b, sq, sk, nq, nkv, d,
                         _strides(q, r), _strides(k, 1)[:3], _strides(k, 1)[:3],
                         [o.stride(0), o.stride(1), o.stride(2)], bool(causal), float(scale),
                         None, None, None, None)
    return dq.float(), dk.float(), dv.float()


def _merge(o, lse, o_j, lse_j):
    """Log-sum-exp combine of two partial attentions ([b, s, n, d], [b, n, s])."""
    if o is None:
        return o_j, lse_j
    new = torch.logaddexp(lse, lse_j)
    w_old = torch.exp(lse - new).permute(0, 2, 1)[..., None]
    w_new = torch.exp(lse_j - new).permute(0, 2, 1)[..., None]
    return o * w_old + o_j * w_new, new


def _visible(j, r, causal):
    """(run the pair?, causal kernel?) for chunk j against local queries of rank r."""
    if not causal:
        return True, False
    return j <= r, j == r


# ---------------------------------------------------------------------------
# ring exchange
# ---------------------------------------------------------------------------
class _Ring:
    """Send to the next rank / receive from the previous one of ``group``."""

    def __init__(self, group):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        ranks = dist.get_process_group_ranks(group)
        self.next = ranks[(self.rank + 1) % self.world]
        self.prev = ranks[(self.rank - 1) % self.world]

    def shift(self, tensors):
        """Post the exchange of ``tensors``; returns (work, received buffers)."""
        recv = [torch.empty_like(t) for t in tensors]
        ops = [("send", t, self.next) for t in tensors] + [("recv", t, self.prev) for t in recv]
        return comm.p2p(ops, group=self.group, async_op=True), recv


class _RingAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, group, causal, scale):
        ring = _Ring(group)
        W, r = ring.world, ring.rank
        o = lse = None
        kv = [k.contiguous(), v.contiguous()]
        for i in range(W):
            j = (r - i) % W
            work = recv = None
            if i + 1 < W:
                work, recv = ring.shift(kv)  # next chunk in flight during this step
            run, c = _visible(j, r, causal)
            if run:
                o_j, lse_j = _pair_fwd(q, kv[0], kv[1], c, scale)
                o, lse = _merge(o, lse, o_j, lse_j)
            if work is not None:
                work.wait()
                kv = recv
        out = o.to(q.dtype)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.group, ctx.causal, ctx.scale = group, causal, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        ring = _Ring(ctx.group)
        W, r = ring.world, ring.rank
        dout = dout.contiguous()
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        # the travelling chunk: K, V and its dK, dV accumulators (fp32)
        buf = [k.contiguous(), v.contiguous(),
               torch.zeros(k.shape, dtype=torch.float32, device=k.device),
               torch.zeros(v.shape, dtype=torch.float32, device=v.device)]
        for i in range(W):
            j = (r - i) % W
            run, c = _visible(j, r, ctx.causal)
            if run:
                dq_j, dk_j, dv_j = _pair_bwd(q, buf[0], buf[1], out, lse, dout, c, ctx.scale)
                dq += dq_j
                buf[2] = buf[2] + dk_j
                buf[3] = buf[3] + dv_j
            if W > 1:  # W hops bring every chunk back to its owner
                work, recv = ring.shift(buf)
                work.wait()
                buf = recv
        return dq.to(q.dtype), buf[2].to(k.dtype), buf[3].to(v.dtype), None, None, None


def ring_attention(q, k, v, group, causal=True, softmax_scale=None):
    """Attention of the local query chunk over the whole sequence of ``group``.

    q ``[b, s, nq, d]``, k / v ``[b, s, nkv, d]``: this rank's contiguous
    sequence chunk (rank r of the group holds positions r*s .. r*s+s-1).
    Returns ``[b, s, nq, d]``."""
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if group is None or dist.get_world_size(group) == 1:
        from ..ops.attention import flash_attn_func
        return flash_attn_func(q, k, v, causal=causal, softmax_scale=scale)
    return _RingAttnFn.apply(q, k, v, group, causal, scale)


def ring_attention_simulated(qs, ks, vs, causal=True, softmax_scale=None, grad_outs=None):
    """The W ranks of a ring run one after another in one process (kernel
    tests on one GPU): ``qs`` / ``ks`` / ``vs`` are the per-rank chunks.
    Returns the per-rank outputs and, with ``grad_outs``, (dq, dk, dv) per rank."""
    W = len(qs)
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(qs[0].shape[-1])
    outs, lses = [], []
    for r in range(W):
        o = lse = None
        for i in range(W):
            j = (r - i) % W
            run, c = _visible(j, r, causal)
            if run:
                o, lse = _merge(o, lse, *_pair_fwd(qs[r], ks[j], vs[j], c, scale))
        outs.append(o.to(qs[r].dtype))
        lses.append(lse)
    if grad_outs is None:
        return outs
    dqs = [torch.zeros(q.shape, dtype=torch.float32, device=q.device) for q in qs]
    dks = [torch.zeros(k.shape, dtype=torch.float32, device=k.device) for k in ks]
    dvs = [torch.zeros(v.shape, dtype=torch.float32, device=v.device) for v in vs]
    for r in range(W):
        for j in range(W):
            run, c = _visible(j, r, causal)
            if run:
                dq, dk, dv = _pair_bwd(qs[r], ks[j], vs[j], outs[r], lses[r], grad_outs[r], c,
                                       scale)
                dqs[r] += dq
                dks[j] += dk
                dvs[j] += dv
    return outs, (dqs, dks, dvs)


# ---------------------------------------------------------------------------
# training integration
# ---------------------------------------------------------------------------
def get_batch_on_this_cp_rank(tensors, dim=1):
    """This rank's contiguous chunk (along the sequence ``dim``) of every tensor."""
    from . import state
    C = state.get_context_parallel_world_size()
    if C == 1:
        return tensors
    r = state.get_context_parallel_rank()
    out = []
    for t in tensors:
        if t is None or not torch.is_tensor(t) or t.dim() <= dim:
            out.append(t)
            continue
        c = t.shape[dim] // C
        out.append(t.narrow(dim, r * c, c).contiguous())
    return out


def cp_token_mean(losses, loss_mask):
    """Masked token mean of the local chunk's ``losses`` scaled so that the DP
    average over the C ranks of a sequence is the whole sequence's mean:
    ``C * sum(local) / sum(mask over the group)``."""
    from . import state
    group = state.get_context_parallel_group()
    if group is None:
        return torch.sum(losses * loss_mask) / loss_mask.sum()
    n = loss_mask.sum().detach().clone()
    comm.all_reduce(n, group=group)
    return torch.sum(losses * loss_mask) * dist.get_world_size(group) / n


def chunk_position_ids(s, b, device):
    """Global positions of this rank's chunk ``[b, s]``."""
    from . import state
    r = state.get_context_parallel_rank()
    return (r * s + torch.arange(s, device=device)).unsqueeze(0).expand(b, s)

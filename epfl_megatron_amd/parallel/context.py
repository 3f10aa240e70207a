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
          values).  dQ stays local.  K/V travel as in the forward (posted
          before the step's kernels); the dK_j / dV_j accumulators follow one
          hop behind: posted after the step's kernels, received and added
          after the NEXT step's kernels, so both transfers overlap compute.
          After W hops every accumulator is back at its owner.

The per-pair kernels are the training kernels (``csrc/flash_attn_fwd.hip`` /
``flash_attn_bwd.hip``: native GQA, LSE in natural log); on CPU tensors the
same math runs in fp32 torch (tests, gloo).  ``ring_attention_simulated`` runs
the W ranks of a ring one after another in one process (kernel-level tests on
one GPU).

Zig-zag layout: with a contiguous split the causal work grows with the rank
(rank W-1 runs W pairs, rank 0 one).  Cutting the sequence into 2W pieces and
giving rank r pieces r and 2W-1-r makes every off-diagonal pair exactly half
a pair (``_plan``), so all ranks finish each ring step together.

Training integration (``--context_parallel_size C``): C consecutive DP ranks
form a context-parallel group (``state.get_context_parallel_group``) and read
the same samples; ``get_batch_on_this_cp_rank`` keeps this rank's zig-zag
share of the sequence (global position ids included), self-attention runs
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


def _visible(b, sq, sk, causal, docs, coff, device):
    """Boolean [b, sq, sk] visibility of a pair (CPU path): key k is seen by
    query q iff k <= q + coff (causal) and k >= docs[0][b, q] (documents)."""
    i = torch.arange(sq, device=device)[:, None]
    j = torch.arange(sk, device=device)[None, :]
    vis = torch.ones(1, sq, sk, dtype=torch.bool, device=device)
    if causal:
        vis = vis & (j <= i + (sk - sq if coff is None else coff))[None]
    if docs is not None:
        vis = vis & (j[None] >= docs[0].long().to(device)[:, :, None])
    return vis.expand(b, sq, sk)


def _pair_fwd(q, k, v, causal, scale, docs=None, coff=None):
    """(O [b, s, nq, d] fp32-accurate in q.dtype, LSE [b, nq, s] fp32 natural log).
    ``docs``: the pair's local document arrays (``_pair_docs``), ``coff`` its
    causal offset (None: sk - sq)."""
    b, sq, nq, d = q.shape
    sk, nkv = k.shape[1], k.shape[2]
    if not q.is_cuda:
        if docs is None and coff is None:
            from ..ops.attention import attention_ref
            o, lse = attention_ref(q, k, v, causal, scale, return_lse=True)
            return o.float(), lse.float()
        r = nq // nkv
        kx = k.float().repeat_interleave(r, dim=2)
        vx = v.float().repeat_interleave(r, dim=2)
        sc = torch.einsum("bqhd,bkhd->bhqk", q.float(), kx) * scale
        vis = _visible(b, sq, sk, causal, docs, coff, q.device)[:, None]
        sc = sc.masked_fill(~vis, float("-inf"))
        lse = torch.logsumexp(sc, -1)  # [b, h, q]; -inf for a row that sees no key
        p = torch.exp(sc - lse[..., None].clamp_min(-1e30))
        o = torch.einsum("bhqk,bkhd->bqhd", p.nan_to_num(0.0), vx)
        return o, lse
    from ..ops._ext import ext
    r = nq // nkv
    out = torch.empty_like(q)
    lse = torch.empty(b, nq, sq, dtype=torch.float32, device=q.device)
    assert docs is None and coff is None, "document pairs run the fused (merge) forward"
    ext().flash_attn_fwd(q, k, v, out, lse, b, sq, sk, nq, nkv, d, _strides(q, r),
                         _strides(k, 1)[:3], _strides(v, 1)[:3],
                         [out.stride(0), out.stride(1), out.stride(2)], bool(causal),
                         float(scale), None, None, None, None)
    return out.float(), lse


def _pair_bwd(q, k, v, o, lse, do, causal, scale, docs=None, coff=None):
    """dQ, dK, dV of one pair given the GLOBAL output ``o`` and ``lse``."""
    b, sq, nq, d = q.shape
    sk, nkv = k.shape[1], k.shape[2]
    r = nq // nkv
    if not q.is_cuda:
        qf, kf, vf, of, dof = (t.float() for t in (q, k, v, o, do))
        kx = kf.repeat_interleave(r, dim=2)
        vx = vf.repeat_interleave(r, dim=2)
        s = torch.einsum("bqhd,bkhd->bhqk", qf, kx) * scale
        if causal or docs is not None:
            vis = _visible(b, sq, sk, causal, docs, coff, q.device)[:, None]
            s = s.masked_fill(~vis, float("-inf"))
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
                         _strides(q, r), _strides(k, 1)[:3], _strides(v, 1)[:3],
                         [o.stride(0), o.stride(1), o.stride(2)], bool(causal), float(scale),
                         None, None, None, docs, -1 if coff is None else int(coff))
    return dq.float(), dk.float(), dv.float()


def _pair_fwd_into(q, k, v, o32, lse, causal, scale, merge, docs=None, coff=None):
    """GPU: one pair's attention log-sum-exp combined IN the kernel epilogue with
    the running fp32 output ``o32`` [b, s, nq, d] and ``lse`` [b, nq, s] (views
    allowed): no O_j / LSE_j tensors and no separate merge kernels."""
    from ..ops._ext import ext
    b, sq, nq, d = q.shape
    sk, nkv = k.shape[1], k.shape[2]
    r = nq // nkv
    ext().flash_attn_fwd_merge(q, k, v, o32, lse, b, sq, sk, nq, nkv, d, _strides(q, r),
                               _strides(k, 1)[:3], _strides(v, 1)[:3], bool(causal), float(scale),
                               bool(merge), docs, -1 if coff is None else int(coff))


def _merge(o, lse, o_j, lse_j):
    """Log-sum-exp combine of two partial attentions ([b, s, n, d], [b, n, s])."""
    if o is None:
        return o_j, lse_j
    new = torch.logaddexp(lse, lse_j)
    w_old = torch.exp(lse - new).permute(0, 2, 1)[..., None]
    w_new = torch.exp(lse_j - new).permute(0, 2, 1)[..., None]
    return o * w_old + o_j * w_new, new


def _plan(j, r, causal, zigzag):
    """Which rows of the local Q and of K/V chunk j meet, and with which mask.

    Returns None (pair fully masked) or (q_rows, kv_rows, causal_kernel) with
    rows ``"all"``, ``"first"`` or ``"second"`` (halves of the chunk).
    zig-zag layout (``zigzag=True``): rank r holds sequence pieces r and
    2W-1-r of 2W, so for causal attention every off-diagonal pair is half a
    pair (j < r: all queries see K/V piece j only; j > r: only the late query
    piece sees both K/V pieces) and all ranks do the same work."""
    if not causal:
        return "all", "all", False
    if j == r:
        return "all", "all", True
    if not zigzag:
        return ("all", "all", False) if j < r else None
    return ("all", "first", False) if j < r else ("second", "all", False)


def _rows(t, which, dim=1):
    if which == "all":
        return t
    h = t.shape[dim] // 2
    return t.narrow(dim, 0, h) if which == "first" else t.narrow(dim, h, t.shape[dim] - h)


# ---------------------------------------------------------------------------
# document masks (--reset_attention_mask) over the ring
# ---------------------------------------------------------------------------
def _positions(rank, world, s, zigzag, device):
    """Global sequence positions of the ``s`` local rows of ``rank``."""
    if zigzag:
        n = s // 2
        lo, hi = rank * n, (2 * world - 1 - rank) * n
        return torch.cat([torch.arange(lo, lo + n, device=device),
                          torch.arange(hi, hi + n, device=device)])
    return torch.arange(rank * s, rank * s + s, device=device)


def _subpairs(plan, docs):
    """With documents every pair runs with sq == sk (the kernels' document
    arrays are square): a half pair (all rows x one piece, or one piece x all)
    splits into its two piece x piece quarters."""
    qs, ks, c = plan
    if docs is None or qs == ks or (qs != "all" and ks != "all"):
        return [plan]
    if qs == "all":
        return [("first", ks, c), ("second", ks, c)]
    return [(qs, "first", c), (qs, "second", c)]


def _pair_docs(docs, pq, pk):
    """Local int32 [2, b, n] document arrays of a pair from the GLOBAL bounds
    ``docs`` [2, b, S] and the pair's (sorted) query / key positions: per query
    the first local key at or after its document start, per key the first local
    query at or after its document end (the kernels' doc_start / doc_end)."""
    start = torch.searchsorted(pk, docs[0][:, pq].long().contiguous())
    end = torch.searchsorted(pq, docs[1][:, pk].long().contiguous())
    return torch.stack([start, end]).to(torch.int32).contiguous()


def _pair_masks(docs, plan, posq, posk):
    """(causal kernel, local doc arrays, causal offset) of one (sub)pair.  With
    documents an off-diagonal pair (every key before every query) runs the
    causal kernel with offset sk: no causal cut, document starts only."""
    qs, ks, c = plan
    if docs is None:
        return c, None, None
    pq, pk = _rows(posq, qs, 0), _rows(posk, ks, 0)
    pd = _pair_docs(docs, pq, pk)
    return (True, pd, None) if c else (True, pd, pk.numel())


def _merge_rows(o, lse, o_j, lse_j, which):
    """``_merge`` into the rows ``which`` of the running (o, lse)."""
    if o is None or which == "all":
        return _merge(o, lse, o_j, lse_j)
    o2, l2 = _merge(_rows(o, which), _rows(lse, which, 2), o_j, lse_j)
    o, lse = o.clone(), lse.clone()
    _rows(o, which).copy_(o2)
    _rows(lse, which, 2).copy_(l2)
    return o, lse


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
    def forward(ctx, q, k, v, group, causal, scale, zigzag, docs):
        ring = _Ring(group)
        W, r = ring.world, ring.rank
        o = lse = None
        fused = q.is_cuda
        if fused:  # running output / lse, merged by the kernels in place
            b, s, nq, d = q.shape
            o = torch.empty(b, s, nq, d, dtype=torch.float32, device=q.device)
            lse = torch.empty(b, nq, s, dtype=torch.float32, device=q.device)
        posq = _positions(r, W, q.shape[1], zigzag, q.device) if docs is not None else None
        started = False
        kv = [k.contiguous(), v.contiguous()]
        for i in range(W):
            j = (r - i) % W
            work = recv = None
            if i + 1 < W:
                work, recv = ring.shift(kv)  # next chunk in flight during this step
            plan = _plan(j, r, causal, zigzag)
            posk = _positions(j, W, k.shape[1], zigzag, q.device) if docs is not None else None
            for sp in ([] if plan is None else _subpairs(plan, docs)):
                qs, ks, _ = sp
                c, pd, coff = _pair_masks(docs, sp, posq, posk)
                if fused:
                    # step 0 is the diagonal ("all" rows): it initialises o / lse
                    _pair_fwd_into(_rows(q, qs), _rows(kv[0], ks), _rows(kv[1], ks),
                                   _rows(o, qs), _rows(lse, qs, 2), c, scale, merge=started,
                                   docs=pd, coff=coff)
                    started = True
                else:
                    o_j, lse_j = _pair_fwd(_rows(q, qs), _rows(kv[0], ks), _rows(kv[1], ks), c,
                                           scale, pd, coff)
                    o, lse = _merge_rows(o, lse, o_j, lse_j, qs)
            if work is not None:
                work.wait()
                kv = recv
        out = o.to(q.dtype)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.group, ctx.causal, ctx.scale, ctx.zigzag, ctx.docs = group, causal, scale, zigzag, docs
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        docs = ctx.docs
        ring = _Ring(ctx.group)
        W, r = ring.world, ring.rank
        dout = dout.contiguous()
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        posq = _positions(r, W, q.shape[1], ctx.zigzag, q.device) if docs is not None else None
        kv = [k.contiguous(), v.contiguous()]
        acc_work = acc_recv = None
        for i in range(W):
            j = (r - i) % W
            kv_work = kv_recv = None
            if i + 1 < W:  # K / V of the next step in flight during this one
                kv_work, kv_recv = ring.shift(kv)
            dk = torch.zeros(k.shape, dtype=torch.float32, device=k.device)
            dv = torch.zeros(v.shape, dtype=torch.float32, device=v.device)
            plan = _plan(j, r, ctx.causal, ctx.zigzag)
            posk = _positions(j, W, k.shape[1], ctx.zigzag, q.device) if docs is not None else None
            for sp in ([] if plan is None else _subpairs(plan, docs)):
                qs, ks, _ = sp
                c, pd, coff = _pair_masks(docs, sp, posq, posk)
                dq_j, dk_j, dv_j = _pair_bwd(_rows(q, qs), _rows(kv[0], ks), _rows(kv[1], ks),
                                             _rows(out, qs), _rows(lse, qs, 2), _rows(dout, qs), c,
                                             ctx.scale, pd, coff)
                _rows(dq, qs).add_(dq_j)
                _rows(dk, ks).add_(dk_j)
                _rows(dv, ks).add_(dv_j)
            if acc_work is not None:  # chunk j's dK / dV so far, sent by the previous rank
                acc_work.wait()
                dk += acc_recv[0]
                dv += acc_recv[1]
            if W > 1:  # travels on while the next pair computes; W hops end at the owner
                acc_work, acc_recv = ring.shift([dk, dv])
            if kv_work is not None:
                kv_work.wait()
                kv = kv_recv
        if acc_work is not None:
            acc_work.wait()
            dk, dv = acc_recv
        return (dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype), None, None, None, None, None)


def ring_attention(q, k, v, group, causal=True, softmax_scale=None, zigzag=False, docs=None):
    """Attention of the local query chunk over the whole sequence of ``group``.

    q ``[b, s, nq, d]``, k / v ``[b, s, nkv, d]``: this rank's sequence chunk,
    contiguous (rank r of W holds positions r*s .. r*s+s-1) or, with
    ``zigzag``, the pieces r and 2W-1-r of 2W (s/2 positions each, in that
    order; ``zigzag_slice``), which balances causal work over the ranks.
    ``docs``: packed-document bounds of the WHOLE sequence, int32 ``[2, b, S]``
    (``utils.misc.doc_bounds``; the same on every rank of the group): keys of
    earlier documents are masked (``--reset_attention_mask``).
    Returns ``[b, s, nq, d]``."""
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if group is None or dist.get_world_size(group) == 1:
        from ..ops.attention import flash_attn_func
        if docs is not None:  # (the model runs flash_attn_qkvpacked with doc bounds here)
            raise ValueError("ring_attention with documents needs a context-parallel group")
        return flash_attn_func(q, k, v, causal=causal, softmax_scale=scale)
    if zigzag and q.shape[1] % 2:
        raise ValueError("zig-zag context parallelism needs an even local chunk")
    if docs is not None:
        if not causal:
            raise ValueError("document masks need causal attention")
        docs = docs.to(device=q.device, dtype=torch.int32).contiguous()
    return _RingAttnFn.apply(q, k, v, group, causal, scale, bool(zigzag), docs)


def zigzag_slice(t, dim, rank, world):
    """Pieces ``rank`` and ``2*world-1-rank`` of ``2*world`` along ``dim``."""
    n = t.shape[dim] // (2 * world)
    return torch.cat([t.narrow(dim, rank * n, n),
                      t.narrow(dim, (2 * world - 1 - rank) * n, n)], dim)


def ring_attention_simulated(qs, ks, vs, causal=True, softmax_scale=None, grad_outs=None,
                             zigzag=False, docs=None):
    """The W ranks of a ring run one after another in one process (kernel
    tests on one GPU): ``qs`` / ``ks`` / ``vs`` are the per-rank chunks,
    ``docs`` the whole sequence's document bounds (as ``ring_attention``).
    Returns the per-rank outputs and, with ``grad_outs``, (dq, dk, dv) per rank."""
    W = len(qs)
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(qs[0].shape[-1])
    dev = qs[0].device
    if docs is not None:
        docs = docs.to(device=dev, dtype=torch.int32).contiguous()
    pos = [_positions(r, W, qs[r].shape[1], zigzag, dev) for r in range(W)] if docs is not None \
        else [None] * W
    outs, lses = [], []
    for r in range(W):
        o = lse = None
        fused = qs[r].is_cuda
        if fused:
            b, s, nq, d = qs[r].shape
            o = torch.empty(b, s, nq, d, dtype=torch.float32, device=dev)
            lse = torch.empty(b, nq, s, dtype=torch.float32, device=dev)
        started = False
        for i in range(W):
            j = (r - i) % W
            plan = _plan(j, r, causal, zigzag)
            for sp in ([] if plan is None else _subpairs(plan, docs)):
                q_, k_, _ = sp
                c, pd, coff = _pair_masks(docs, sp, pos[r], pos[j])
                if fused:
                    _pair_fwd_into(_rows(qs[r], q_), _rows(ks[j], k_), _rows(vs[j], k_),
                                   _rows(o, q_), _rows(lse, q_, 2), c, scale, merge=started,
                                   docs=pd, coff=coff)
                    started = True
                    continue
                o_j, lse_j = _pair_fwd(_rows(qs[r], q_), _rows(ks[j], k_), _rows(vs[j], k_), c,
                                       scale, pd, coff)
                o, lse = _merge_rows(o, lse, o_j, lse_j, q_)
        outs.append(o.to(qs[r].dtype))
        lses.append(lse)
    if grad_outs is None:
        return outs
    dqs = [torch.zeros(q.shape, dtype=torch.float32, device=q.device) for q in qs]
    dks = [torch.zeros(k.shape, dtype=torch.float32, device=k.device) for k in ks]
    dvs = [torch.zeros(v.shape, dtype=torch.float32, device=v.device) for v in vs]
    for r in range(W):
        for j in range(W):
            plan = _plan(j, r, causal, zigzag)
            for sp in ([] if plan is None else _subpairs(plan, docs)):
                q_, k_, _ = sp
                c, pd, coff = _pair_masks(docs, sp, pos[r], pos[j])
                dq, dk, dv = _pair_bwd(_rows(qs[r], q_), _rows(ks[j], k_), _rows(vs[j], k_),
                                       _rows(outs[r], q_), _rows(lses[r], q_, 2),
                                       _rows(grad_outs[r], q_), c, scale, pd, coff)
                _rows(dqs[r], q_).add_(dq)
                _rows(dks[j], k_).add_(dk)
                _rows(dvs[j], k_).add_(dv)
    return outs, (dqs, dks, dvs)


# ---------------------------------------------------------------------------
# training integration
# ---------------------------------------------------------------------------
def get_batch_on_this_cp_rank(tensors, dim=1):
    """This rank's zig-zag share (``zigzag_slice``) along the sequence ``dim``."""
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
        out.append(zigzag_slice(t, dim, r, C).contiguous())
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
    """Global positions ``[b, s]`` of this rank's zig-zag share of ``s`` rows."""
    from . import state
    C = state.get_context_parallel_world_size()
    r = state.get_context_parallel_rank()
    full = torch.arange(s * C, device=device)
    return zigzag_slice(full, 0, r, C).unsqueeze(0).expand(b, s)

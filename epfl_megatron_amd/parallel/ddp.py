"""Data-parallel gradient reduction: contiguous buffers, buckets, overlap.

Reference ``megatron/model/distributed.py`` keeps one contiguous fp32 gradient
buffer and issues ONE all-reduce of the whole buffer after the entire backward
(``distributed.py:202-209``).  On MI355X that serialises a 27 GB
collective (Llama-2-7B, DP=8) behind the backward pass.  This implementation
keeps the contiguous fp32 buffer (so ``param.main_grad`` views and the fused
wgrad GEMM still work) but cuts it into buckets in reverse parameter order —
the order gradients become ready — and launches each bucket's RCCL collective
as soon as its last gradient has been produced, overlapping DP communication
with the rest of the backward.  Bucket size (``--ddp_bucket_size_mb``) is the
knob for the xGMI mesh: large enough that each ring collective is
bandwidth-bound on the 7 links, small enough that the exposed tail (the first
layers + embedding) stays short.

The same layout carries a contiguous buffer of the model's (bf16) parameters:
every parameter's ``.data`` is re-pointed into it, so the optimizer updates
all parameters with ONE flat streaming kernel and the distributed optimizer
all-gathers parameter shards bucket by bucket.

With ``use_distributed_optimizer`` each bucket is padded to a multiple of the
DP size and reduce-scattered in place (rank r owns bucket slice r); after the
optimizer step the bf16 parameter shards are all-gathered back ASYNCHRONOUSLY
(``start_param_sync``): forward pre-hooks wait only for the bucket holding the
parameters a module is about to use, so the gather overlaps the next forward
(reference gathers synchronously, ``distrib_optimizer.py:571-600``).

Correctness rules the bucket logic enforces (all collectives go through
``comm``, the same calls on RCCL and on the gloo test path):

* a bucket is launched only after EVERY gradient contribution to it has been
  written.  Parameters with several contributions (the tied word embedding:
  lookup + LM head) or with a cross-stage reduction that must precede the DP
  reduction (tied embeddings / T5 position embeddings at PP > 1, reference
  ``optimizer.py:203-254``) are "held": they live in a trailing bucket that is
  launched only by ``start_grad_sync`` after the optimizer has done those
  reductions;
* nothing writes a bucket between its launch and ``wait`` (checked by
  ``EMA_COMM_CHECK=1``).
"""
import contextlib

import torch
import torch.distributed as dist

from . import state, comm

_ALIGN = 64  # elements; keeps every param view 128/256-byte aligned


def _round_up(x, m):
    return (x + m - 1) // m * m


class Bucket:
    __slots__ = ("index", "start", "end", "params", "pending", "handle", "shard_size", "held")

    def __init__(self, index, start, end, params, shard_size, held=False):
        self.index = index
        self.start = start
        self.end = end
        self.params = params
        self.pending = 0
        self.handle = None
        self.shard_size = shard_size
        self.held = held

    @property
    def numel(self):
        return self.end - self.start


def _unwrap(module):
    m = module
    while hasattr(m, "module") and isinstance(m.module, torch.nn.Module):
        m = m.module
    return m


def held_parameters(module):
    """Parameters whose DP reduction must wait for ``start_grad_sync``: tied word
    embeddings (two contributions; embedding-group all-reduce at PP > 1) and the
    T5 split-rank position embeddings."""
    m = _unwrap(module)
    held = [p for p in m.parameters() if getattr(p, "_ddp_hold", False)]
    if getattr(m, "share_word_embeddings", False) and hasattr(m, "word_embeddings_weight"):
        lm = getattr(m, "language_model", None)
        tied = lm is None or getattr(lm, "tie_embed_logits", True)
        try:
            w = m.word_embeddings_weight()
        except Exception:  # stage without an embedding
            w = None
        if tied and w is not None and w.requires_grad:
            held.append(w)
    lm = getattr(m, "language_model", None)
    emb = getattr(lm, "embedding", None) if lm is not None else None
    pe = getattr(emb, "position_embeddings", None) if emb is not None else None
    if pe is not None and state.get_pipeline_model_parallel_split_rank() is not None \
            and state.get_pipeline_model_parallel_world_size() > 1:
        held.append(pe.weight)
    seen, out = set(), []
    for p in held:
        if id(p) not in seen:
            seen.add(id(p))
            out.append(p)
    return out


def late_use_parameters(module):
    """Parameters used at the END of the forward although they are attributes of
    an outer module (untied ``lm_head``, last-stage tied embedding copy): their
    all-gather wait happens in ``word_embeddings_weight()``, not in the owning
    module's pre-hook (which would block the whole forward)."""
    m = _unwrap(module)
    out = []
    lm = getattr(m, "language_model", None)
    if lm is not None and isinstance(getattr(lm, "lm_head", None), torch.nn.Parameter):
        out.append(lm.lm_head)
    we = getattr(m, "word_embeddings", None)
    if we is not None and getattr(we, "weight", None) is not None:
        out.append(we.weight)
    return out


class DistributedDataParallel(torch.nn.Module):
    def __init__(self, module, accumulate_allreduce_grads_in_fp32=True,
                 use_contiguous_buffers=True, bucket_size_mb=256.0, overlap_grad_reduce=True,
                 use_distributed_optimizer=False, data_parallel_group=None,
                 overlap_param_gather=True):
        super().__init__()
        if not use_contiguous_buffers:
            raise AssertionError("the MI355X DDP always uses contiguous buffers")
        self.module = module
        self.dp_group = data_parallel_group if data_parallel_group is not None \
            else state.get_data_parallel_group()
        # bucket i reduces / gathers on comm_groups[i % n] (own RCCL stream each)
        self.comm_groups = [self.dp_group] if data_parallel_group is not None \
            else state.get_data_parallel_comm_groups()
        self.dp_size = dist.get_world_size(self.dp_group)
        self.dp_rank = dist.get_rank(self.dp_group)
        self.overlap = overlap_grad_reduce and self.dp_size > 1
        self.use_distributed_optimizer = use_distributed_optimizer
        self.bucket_size_mb = bucket_size_mb
        self._sync_enabled = True

        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise AssertionError("model has no trainable parameters")
        pdtype = params[0].dtype
        for p in params:
            if p.dtype != pdtype:
                raise AssertionError("all parameters must share one dtype")
        self.param_dtype = pdtype
        self.grad_dtype = torch.float32 if accumulate_allreduce_grads_in_fp32 else pdtype
        device = params[0].device
        held_ids = {id(p) for p in held_parameters(module)}
        self.held = [p for p in params if id(p) in held_ids]

        # ---- layout: reverse param order, aligned, cut into buckets; held
        # params in one trailing bucket -------------------------------------
        bucket_elems = max(int(bucket_size_mb * 1024 * 1024 / 4), _ALIGN)
        pad_unit = _ALIGN * (self.dp_size if use_distributed_optimizer else 1)
        offsets = {}
        buckets_spec = []
        cur, cur_params, bstart = 0, [], 0
        for p in reversed(params):
            if id(p) in held_ids:
                continue
            cur = _round_up(cur, _ALIGN)
            offsets[p] = cur
            cur += p.numel()
            cur_params.append(p)
            if cur - bstart >= bucket_elems:
                end = _round_up(cur, pad_unit)
                buckets_spec.append((bstart, end, cur_params, False))
                cur, bstart, cur_params = end, end, []
        if cur_params:
            end = _round_up(cur, pad_unit)
            buckets_spec.append((bstart, end, cur_params, False))
            cur = bstart = end
        if self.held:
            cur_params = []
            for p in reversed(self.held):
                cur = _round_up(cur, _ALIGN)
                offsets[p] = cur
                cur += p.numel()
                cur_params.append(p)
            end = _round_up(cur, pad_unit)
            buckets_spec.append((bstart, end, cur_params, True))
            cur = end
        total = cur
        self.numel = total
        self.param_index = {}
        self.grad_buffer = torch.zeros(total, dtype=self.grad_dtype, device=device)
        self.param_buffer = torch.zeros(total, dtype=pdtype, device=device)
        for p in params:
            off = offsets[p]
            n = p.numel()
            self.param_index[p] = (off, n)
            pv = self.param_buffer[off:off + n].view_as(p)
            pv.copy_(p.data)
            p.data = pv
            p.main_grad = self.grad_buffer[off:off + n].view_as(p)
        self.buckets = []
        self._param_bucket = {}
        for i, (s, e, ps, held) in enumerate(buckets_spec):
            shard = (e - s) // self.dp_size if use_distributed_optimizer else 0
            b = Bucket(i, s, e, ps, shard, held)
            self.buckets.append(b)
            for p in ps:
                self._param_bucket[p] = b
        self._hooks = []
        for p in params:
            p._main_grad_ready = self._make_ready_cb(p)
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_accum_hook(p)))
        self._reset_pending()

        # ---- async dist-opt parameter all-gather --------------------------
        self.overlap_param_gather = (overlap_param_gather and use_distributed_optimizer
                                     and self.dp_size > 1)
        self._ag_handles = []   # Work objects in issue order
        self._ag_pos = {}       # bucket index -> position in issue order
        self._ag_done = 0
        if self.overlap_param_gather:
            late = {id(p) for p in late_use_parameters(module)}
            for mod in module.modules():
                own = [p for p in mod.parameters(recurse=False)
                       if p.requires_grad and id(p) not in late and p in self._param_bucket]
                if own:
                    idx = sorted({self._param_bucket[p].index for p in own})
                    self._hooks.append(mod.register_forward_pre_hook(self._make_ag_hook(idx)))
            for p in params:
                p._param_sync_wait = self._make_param_wait(p)

    # ---- gradient hooks ----------------------------------------------------
    def _reset_pending(self):
        for b in self.buckets:
            b.pending = len(b.params)
            b.handle = None
        self._seen = set()

    def _make_accum_hook(self, p):
        def hook(param):
            if param.grad is not None:
                g = param.grad.view_as(param.main_grad)
                if getattr(param, "_mg_fresh", False):
                    param.main_grad.copy_(g)
                    param._mg_fresh = False
                else:
                    param.main_grad.add_(g)
                param.grad = None
            self._mark_ready(param)
        return hook

    def _zero_untouched(self, params=None):
        """main_grad of params that got no gradient this step (still fresh) -> 0."""
        for p in (self.param_index if params is None else params):
            if getattr(p, "_mg_fresh", False):
                p.main_grad.zero_()
                p._mg_fresh = False

    def _make_ready_cb(self, p):
        def cb():
            self._mark_ready(p)
        return cb

    def _mark_ready(self, p):
        if not (self.overlap and self._sync_enabled):
            return
        b = self._param_bucket[p]
        if b.held or p in self._seen:
            return
        self._seen.add(p)
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    # ---- collectives -------------------------------------------------------
    def _launch(self, b):
        data = self.grad_buffer[b.start:b.end]
        grp = self.comm_groups[b.index % len(self.comm_groups)]
        # RCCL averages inside the reduction (ncclAvg): no separate 1/dp pass.
        if self.use_distributed_optimizer:
            out = data[self.dp_rank * b.shard_size:(self.dp_rank + 1) * b.shard_size]
            b.handle = comm.reduce_scatter_into(out, data, group=grp, op="avg", async_op=True)
        else:
            b.handle = comm.all_reduce(data, group=grp, op="avg", async_op=True)
        b.pending = -1  # launched

    def start_grad_sync(self):
        """Launch every bucket not launched yet (held buckets included)."""
        if self.dp_size == 1:
            return
        self.wait_param_sync()
        for b in self.buckets:
            if b.pending != -1:
                self._zero_untouched(b.params)
                self._launch(b)

    def finish_grad_sync(self):
        """Launch any bucket not yet launched, then wait for all of them."""
        if self.dp_size == 1:
            self._zero_untouched()
            self._reset_pending()
            return
        self.start_grad_sync()
        for b in self.buckets:
            if b.handle is not None:
                b.handle.wait()
        self._reset_pending()

    # Reference API name.
    def allreduce_gradients(self):
        self.finish_grad_sync()

    @contextlib.contextmanager
    def no_sync(self):
        prev = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = prev

    def set_grad_sync(self, enabled):
        self._sync_enabled = enabled

    def zero_grad_buffer(self):
        """Lazy zeroing: mark every main_grad "fresh".  The first contribution of
        the step then overwrites instead of accumulating (the wgrad GEMM stores
        with beta = 0, hooks copy), and params that receive no gradient are
        zeroed before their bucket is reduced — no 4-bytes/param fill pass."""
        for p in self.param_index:
            p._mg_fresh = True
        self._reset_pending()

    def broadcast_params(self):
        src = state.get_data_parallel_src_rank()
        comm.broadcast(self.param_buffer, src=src, group=self.dp_group)

    # ---- dist-opt parameter all-gather -------------------------------------
    def start_param_sync(self):
        """Dist-opt: every rank updated its shard of each bucket; gather them.
        Issued last bucket first (= forward order); waited lazily by the
        forward pre-hooks when ``overlap_param_gather``, else right here."""
        if not self.use_distributed_optimizer or self.dp_size == 1:
            return
        self.wait_param_sync()
        self._ag_handles, self._ag_pos, self._ag_done = [], {}, 0
        for b in reversed(self.buckets):
            full = self.param_buffer[b.start:b.end]
            mine = full[self.dp_rank * b.shard_size:(self.dp_rank + 1) * b.shard_size]
            self._ag_pos[b.index] = len(self._ag_handles)
            grp = self.comm_groups[b.index % len(self.comm_groups)]
            self._ag_handles.append(comm.all_gather_into(full, mine, group=grp, async_op=True))
        if not self.overlap_param_gather:
            self.wait_param_sync()

    def all_gather_params(self):
        self.start_param_sync()
        self.wait_param_sync()

    def _wait_param_upto(self, pos):
        hs = self._ag_handles
        while self._ag_done <= pos and self._ag_done < len(hs):
            hs[self._ag_done].wait()
            self._ag_done += 1
        if hs and self._ag_done >= len(hs):
            self._ag_handles, self._ag_pos, self._ag_done = [], {}, 0

    def wait_param_sync(self):
        if self._ag_handles:
            self._wait_param_upto(len(self._ag_handles) - 1)

    def _make_ag_hook(self, bucket_indices):
        def hook(_mod, _inp):
            if self._ag_handles:
                pos = max(self._ag_pos.get(i, -1) for i in bucket_indices)
                if pos >= self._ag_done:
                    self._wait_param_upto(pos)
        return hook

    def _make_param_wait(self, p):
        bi = self._param_bucket[p].index

        def wait():
            if self._ag_handles:
                pos = self._ag_pos.get(bi, -1)
                if pos >= self._ag_done:
                    self._wait_param_upto(pos)
        return wait

    def shard_ranges(self):
        """[(bucket_start, shard_offset_in_buffer, shard_len)] owned by this rank."""
        if not self.use_distributed_optimizer:
            return [(0, 0, self.numel)]
        return [(b.start, b.start + self.dp_rank * b.shard_size, b.shard_size)
                for b in self.buckets]

    def layout_signature(self):
        """Everything the flat optimizer-state layout depends on."""
        return {"dp_size": self.dp_size, "numel": self.numel,
                "buckets": [(b.start, b.end) for b in self.buckets],
                "distributed": self.use_distributed_optimizer}

    # ---- module passthrough ------------------------------------------------
    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)

    def state_dict(self, prefix="", keep_vars=False, **kw):
        self.wait_param_sync()
        return self.module.state_dict(prefix=prefix, keep_vars=keep_vars)

    def state_dict_for_save_checkpoint(self, prefix="", keep_vars=False):
        self.wait_param_sync()
        return self.module.state_dict_for_save_checkpoint(prefix=prefix, keep_vars=keep_vars)

    def load_state_dict(self, state_dict, strict=True):
        self.wait_param_sync()
        self.module.load_state_dict(state_dict, strict=strict)

    def set_input_tensor(self, input_tensor):
        return self.module.set_input_tensor(input_tensor)

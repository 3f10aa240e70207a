"""Data-parallel gradient reduction: contiguous buffers, buckets, overlap.

Reference ``megatron/model/distributed.py`` keeps one contiguous fp32 gradient
buffer and issues ONE all-reduce of the whole buffer after the entire backward
(SURVEY D8).  On MI355X that serialises a 27 GB collective (Llama-2-7B, DP=8)
behind the backward pass.  This implementation keeps the contiguous fp32
buffer (so ``param.main_grad`` views and the fused wgrad GEMM still work) but
cuts it into buckets in reverse parameter order — the order gradients become
ready — and launches each bucket's RCCL collective as soon as its last
gradient has been produced, overlapping DP communication with the rest of the
backward.  Bucket size (``--ddp_bucket_size_mb``) is the knob for the xGMI
mesh: large enough that each ring collective is bandwidth-bound on the
7 links, small enough that the exposed tail (the first layers + embedding)
stays short.

The same layout carries a contiguous buffer of the model's (bf16) parameters:
every parameter's ``.data`` is re-pointed into it, so the optimizer updates
all parameters with ONE flat streaming kernel and the distributed optimizer
all-gathers parameter shards bucket by bucket.

With ``use_distributed_optimizer`` each bucket is padded to a multiple of the
DP size and reduce-scattered in place (rank r owns bucket slice r).
"""
import contextlib
import math

import torch
import torch.distributed as dist

from . import state, comm

_ALIGN = 64  # elements; keeps every param view 128/256-byte aligned


def _round_up(x, m):
    return (x + m - 1) // m * m


class Bucket:
    __slots__ = ("index", "start", "end", "params", "pending", "handle", "shard_size")

    def __init__(self, index, start, end, params, shard_size):
        self.index = index
        self.start = start
        self.end = end
        self.params = params
        self.pending = 0
        self.handle = None
        self.shard_size = shard_size

    @property
    def numel(self):
        return self.end - self.start


class DistributedDataParallel(torch.nn.Module):
    def __init__(self, module, accumulate_allreduce_grads_in_fp32=True,
                 use_contiguous_buffers=True, bucket_size_mb=256.0, overlap_grad_reduce=True,
                 use_distributed_optimizer=False, data_parallel_group=None):
        super().__init__()
        if not use_contiguous_buffers:
            raise AssertionError("the MI355X DDP always uses contiguous buffers")
        self.module = module
        self.dp_group = data_parallel_group if data_parallel_group is not None \
            else state.get_data_parallel_group()
        self.dp_size = dist.get_world_size(self.dp_group)
        self.dp_rank = dist.get_rank(self.dp_group)
        self.overlap = overlap_grad_reduce and self.dp_size > 1
        self.use_distributed_optimizer = use_distributed_optimizer
        self._sync_enabled = True
        self._is_gloo = dist.get_backend(self.dp_group) == "gloo"

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

        # ---- layout: reverse param order, aligned, cut into buckets --------
        bucket_elems = max(int(bucket_size_mb * 1024 * 1024 / 4), _ALIGN)
        pad_unit = _ALIGN * (self.dp_size if use_distributed_optimizer else 1)
        offsets = {}
        buckets_spec = []
        cur, cur_params, bstart = 0, [], 0
        for p in reversed(params):
            cur = _round_up(cur, _ALIGN)
            offsets[p] = cur
            cur += p.numel()
            cur_params.append(p)
            if cur - bstart >= bucket_elems:
                end = _round_up(cur, pad_unit)
                buckets_spec.append((bstart, end, cur_params))
                cur, bstart, cur_params = end, end, []
        if cur_params:
            end = _round_up(cur, pad_unit)
            buckets_spec.append((bstart, end, cur_params))
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
        for i, (s, e, ps) in enumerate(buckets_spec):
            shard = (e - s) // self.dp_size if use_distributed_optimizer else 0
            b = Bucket(i, s, e, ps, shard)
            self.buckets.append(b)
            for p in ps:
                self._param_bucket[p] = b
        self._hooks = []
        for p in params:
            p._main_grad_ready = self._make_ready_cb(p)
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_accum_hook(p)))
        self._reset_pending()

    # ---- hooks -----------------------------------------------------------
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
        if p in self._seen:
            return
        self._seen.add(p)
        b = self._param_bucket[p]
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    # ---- collectives -----------------------------------------------------
    def _bucket_view(self, b):
        return self.grad_buffer[b.start:b.end]

    def _launch(self, b):
        data = self._bucket_view(b)
        # RCCL averages in the reduction itself (ncclAvg): no separate 1/dp pass
        # over the bucket.  gloo has no AVG: pre-divide there.
        if self._is_gloo:
            data.div_(self.dp_size)
            op = dist.ReduceOp.SUM
        else:
            op = dist.ReduceOp.AVG
        if self.use_distributed_optimizer:
            out = data[self.dp_rank * b.shard_size:(self.dp_rank + 1) * b.shard_size]
            if self._is_gloo:
                comm.reduce_scatter_into(out, data, group=self.dp_group)
                b.handle = None
            else:
                b.handle = dist.reduce_scatter_tensor(out, data, op=op, group=self.dp_group,
                                                      async_op=True)
        else:
            b.handle = dist.all_reduce(data, op=op, group=self.dp_group,
                                       async_op=not self._is_gloo)
            if self._is_gloo:
                b.handle = None
        b.pending = -1  # launched

    def finish_grad_sync(self):
        """Launch any bucket not yet launched, then wait for all of them."""
        if self.dp_size == 1:
            self._zero_untouched()
            self._reset_pending()
            return
        for b in self.buckets:
            if b.pending != -1:
                self._zero_untouched(b.params)
                self._launch(b)
        for b in self.buckets:
            if b.handle is not None:
                b.handle.wait()
        self._reset_pending()

    # Reference API names.
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
        dist.broadcast(self.param_buffer, src=src, group=self.dp_group)

    def all_gather_params(self):
        """Dist-opt: every rank updated its shard of each bucket; gather them."""
        if not self.use_distributed_optimizer or self.dp_size == 1:
            return
        handles = []
        for b in self.buckets:
            full = self.param_buffer[b.start:b.end]
            mine = full[self.dp_rank * b.shard_size:(self.dp_rank + 1) * b.shard_size]
            if self._is_gloo:
                comm.all_gather_into(full, mine.clone(), group=self.dp_group)
            else:
                handles.append(dist.all_gather_into_tensor(full, mine, group=self.dp_group,
                                                           async_op=True))
        for h in handles:
            h.wait()

    def shard_ranges(self):
        """[(bucket_start, shard_offset_in_buffer, shard_len)] owned by this rank."""
        if not self.use_distributed_optimizer:
            return [(0, 0, self.numel)]
        return [(b.start, b.start + self.dp_rank * b.shard_size, b.shard_size)
                for b in self.buckets]

    # ---- module passthrough ---------------------------------------------
    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)

    def state_dict(self, prefix="", keep_vars=False, **kw):
        return self.module.state_dict(prefix=prefix, keep_vars=keep_vars)

    def state_dict_for_save_checkpoint(self, prefix="", keep_vars=False):
        return self.module.state_dict_for_save_checkpoint(prefix=prefix, keep_vars=keep_vars)

    def load_state_dict(self, state_dict, strict=True):
        self.module.load_state_dict(state_dict, strict=strict)

    def set_input_tensor(self, input_tensor):
        return self.module.set_input_tensor(input_tensor)

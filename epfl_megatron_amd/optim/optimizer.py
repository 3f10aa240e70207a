"""Mixed-precision (and fp32) optimizer over flat DDP buffers, with optional
ZeRO-1 sharding (distributed optimizer).

Behaviour follows the reference (``megatron/optimizer/optimizer.py``,
``distrib_optimizer.py``, ``clip_grads.py``): fp32 master weights for
bf16/fp16 params, grads from the fp32 ``main_grad`` buffer, fp16 loss-scale
unscale + inf check, global L2 grad clipping over non-duplicated params summed
across the model-parallel group (world group with the distributed
optimizer), skip the step on a non-finite grad norm, AdamW (apex FusedAdam
math) or SGD, write back to the model params.

MI355X layout: everything is flat.  Per DDP chunk we keep fp32
``master / exp_avg / exp_avg_sq`` buffers covering the rank's owned ranges of
the gradient buffer (all of it, or its shard of every bucket with the
distributed optimizer) and run ONE fused HIP kernel per step that reads the
grad, applies scale/clip, updates Adam state and master, and writes the bf16
parameter buffer — replacing the reference's copy-grads, unscale, clip,
multi-tensor Adam and copy-back passes.

No host synchronisation per step: the grad norm, clip coefficient, non-finite
flag and Adam step count stay on the device (``step_prep``); the Adam kernel
reads them from device memory and turns itself into a no-op on a non-finite
norm.  ``step()`` returns a :class:`StepResult` whose host values are copied
asynchronously and read lazily (by the log line, one iteration later).  The
LR scheduler is advanced optimistically and rolled back when a step turns out
to have been skipped (resolved before the next step uses the LR).

Checkpoint formats are the reference's: the apex-FusedAdam state_dict
(+ ``fp32_from_fp16_params``) without sharding, and with the distributed
optimizer the per-DP-rank ``optimizer`` + ``shard_fp32_from_float16_groups``
of ``distrib_optimizer.py:415-425``, with shards cut by the REFERENCE's buffer
layout (forward param order packed from the buffer end, one contiguous range
per DP rank, ``distributed.py:130-157`` / ``distrib_optimizer.py:119-164``) —
independent of this framework's bucket layout, so state written at any
``--ddp_bucket_size_mb`` (or by the reference) loads at any other, and at any
DP size.
"""
import math

import torch
import torch.distributed as dist

from ..ops import decode_pack
from ..parallel import state, comm
from ..parallel.tensor.layers import param_is_not_tensor_parallel_duplicate
from ..models.module import param_is_not_shared
from ..ops import optim_kernels as K


class _ChunkState:
    """Flat optimizer state for one DDP model chunk."""

    def __init__(self, ddp, group_of_param, kind):
        self.ddp = ddp
        ranges = ddp.shard_ranges()
        self.numel = sum(n for _, _, n in ranges)
        device = ddp.grad_buffer.device
        self.half_params = ddp.param_dtype != torch.float32
        self.sharded = ddp.use_distributed_optimizer
        # master offset for each owned buffer range
        self.ranges = []
        m = 0
        for _, off, n in ranges:
            self.ranges.append((m, off, n))
            m += n
        if self.half_params or self.sharded:
            self.master = torch.empty(self.numel, dtype=torch.float32, device=device)
            for m_off, b_off, n in self.ranges:
                self.master[m_off:m_off + n].copy_(ddp.param_buffer[b_off:b_off + n])
            self.model_out = ddp.param_buffer
        else:
            self.master = ddp.param_buffer
            self.model_out = None
        self.states = {}
        if kind == "adam":
            self.exp_avg = torch.zeros(self.numel, dtype=torch.float32, device=device)
            self.exp_avg_sq = torch.zeros(self.numel, dtype=torch.float32, device=device)
            self.states = {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq}
        else:
            self.momentum = torch.zeros(self.numel, dtype=torch.float32, device=device)
            self.states = {"momentum_buffer": self.momentum}
        # segments: intersection of each param's [off, off+n) with the owned ranges
        segs = []
        self.param_master_ranges = {}  # p -> [(master_off, param_elem_off, len)]
        for p, (off, n) in ddp.param_index.items():
            g = group_of_param[p]
            count = param_is_not_shared(p) and param_is_not_tensor_parallel_duplicate(p)
            for m_off, b_off, rn in self.ranges:
                lo = max(off, b_off)
                hi = min(off + n, b_off + rn)
                if lo < hi:
                    segs.append((m_off + (lo - b_off), lo, hi - lo, g, count))
                    self.param_master_ranges.setdefault(p, []).append(
                        (m_off + (lo - b_off), lo - off, hi - lo))
        segs.sort(key=lambda t: t[0])
        self.plan = K.ChunkPlan(segs, device)

    def reload_master_from_params(self):
        if self.model_out is None:
            return
        for m_off, b_off, n in self.ranges:
            self.master[m_off:m_off + n].copy_(self.ddp.param_buffer[b_off:b_off + n])

    # -- element-range access (param element coordinates) ------------------
    def read_param_range(self, flat, p, lo, hi, out):
        """Copy the owned part of p.flat[lo:hi] from ``flat`` into out[...] (same coords)."""
        for m_off, p_off, n in self.param_master_ranges.get(p, []):
            a, b = max(lo, p_off), min(hi, p_off + n)
            if a < b:
                out[a - lo:b - lo].copy_(flat[m_off + (a - p_off):m_off + (b - p_off)])

    def write_param_range(self, flat, p, lo, values):
        hi = lo + values.numel()
        for m_off, p_off, n in self.param_master_ranges.get(p, []):
            a, b = max(lo, p_off), min(hi, p_off + n)
            if a < b:
                flat[m_off + (a - p_off):m_off + (b - p_off)].copy_(values[a - lo:b - lo])


class LazyScalar:
    """A host scalar that is read from the device only when first used."""

    __slots__ = ("_fn", "_v")

    def __init__(self, fn):
        self._fn, self._v = fn, None

    def value(self):
        if self._fn is not None:
            self._v, self._fn = self._fn(), None
        return self._v

    def __float__(self):
        return float(self.value())

    def __int__(self):
        return int(self.value())

    def __index__(self):
        return int(self.value())

    def __bool__(self):
        return bool(self.value())

    def __format__(self, spec):
        return format(self.value(), spec)

    def __repr__(self):
        return repr(self.value())

    def __eq__(self, o):
        return self.value() == (o.value() if isinstance(o, LazyScalar) else o)

    def __hash__(self):
        return hash(self.value())

    def __lt__(self, o):
        return self.value() < float(o)

    def __gt__(self, o):
        return self.value() > float(o)

    def __add__(self, o):
        return self.value() + (o.value() if isinstance(o, LazyScalar) else o)

    __radd__ = __add__

    def __sub__(self, o):
        return self.value() - (o.value() if isinstance(o, LazyScalar) else o)

    def __rsub__(self, o):
        return o - self.value()

    def __mul__(self, o):
        return self.value() * (o.value() if isinstance(o, LazyScalar) else o)

    __rmul__ = __mul__

    def __truediv__(self, o):
        return self.value() / (o.value() if isinstance(o, LazyScalar) else o)

    def __abs__(self):
        return abs(self.value())

    def __neg__(self):
        return -self.value()


class StepResult:
    """Device->host mailbox of one optimizer step ([scale, found_inf, step, norm])."""

    def __init__(self, st):
        self._event = None
        if st.is_cuda:
            self._host = torch.empty(st.numel(), dtype=torch.float32, pin_memory=True)
            self._host.copy_(st, non_blocking=True)
            self._event = torch.cuda.Event()
            self._event.record()
        else:
            self._host = st.detach().clone()
        self.sched = None  # (scheduler, increment) applied optimistically
        self.resolved = False

    def _vals(self):
        if self._event is not None:
            self._event.synchronize()
            self._event = None
        return self._host

    @property
    def found_inf(self):
        return bool(self._vals()[1].item() != 0.0)

    @property
    def grad_norm(self):
        return float(self._vals()[3].item())

    @property
    def step(self):
        return int(round(float(self._vals()[2].item())))

    def __bool__(self):  # "update_successful"
        return not self.found_inf


class MegatronOptimizer:
    """Flat-buffer optimizer for a list of DDP-wrapped model chunks."""

    def __init__(self, models, param_groups, kind, lr, weight_decay, adam_beta1=0.9,
                 adam_beta2=0.999, adam_eps=1e-8, sgd_momentum=0.9, clip_grad=0.0,
                 log_num_zeros_in_grad=False, grad_scaler=None, use_distributed_optimizer=False):
        self.models = models
        self.kind = kind
        self.clip_grad = clip_grad
        self.log_num_zeros_in_grad = log_num_zeros_in_grad
        self.grad_scaler = grad_scaler
        self.use_distributed_optimizer = use_distributed_optimizer
        self.beta1, self.beta2, self.eps = adam_beta1, adam_beta2, adam_eps
        self.sgd_momentum = sgd_momentum
        self.param_groups = []
        group_of_param = {}
        for gi, g in enumerate(param_groups):
            pg = {"params": list(g["params"]), "lr": lr, "weight_decay": weight_decay,
                  "wd_mult": g.get("wd_mult", 1.0), "lr_mult": g.get("lr_mult", 1.0),
                  "bias_correction": True, "betas": (adam_beta1, adam_beta2), "eps": adam_eps,
                  "amsgrad": False, "step": 0}
            if kind != "adam":
                pg = {"params": pg["params"], "lr": lr, "weight_decay": weight_decay,
                      "wd_mult": pg["wd_mult"], "lr_mult": pg["lr_mult"],
                      "momentum": sgd_momentum, "dampening": 0, "nesterov": False}
            self.param_groups.append(pg)
            for p in pg["params"]:
                group_of_param[p] = gi
        self._group_of_param = group_of_param
        self.chunks = [_ChunkState(m, group_of_param, kind) for m in models]
        dev = self.chunks[0].master.device
        # [scale, found_inf, step, grad_norm] on the device
        self._st = torch.zeros(4, dtype=torch.float32, device=dev)
        self._host_step = 0          # step count as known on the host (lags when lazy)
        self._pending = None         # StepResult of the last step
        self.found_inf = False

    @property
    def _step(self):
        return int(round(float(self._st[2].item())))

    # -- reference API -------------------------------------------------------
    def zero_grad(self, set_to_none=True):
        for m in self.models:
            m.zero_grad_buffer()
            for p in m.module.parameters():
                p.grad = None

    def get_loss_scale(self):
        if self.grad_scaler is None:
            dev = self.chunks[0].master.device
            return torch.ones((), dtype=torch.float32, device=dev)
        return self.grad_scaler.scale

    def scale_loss(self, loss):
        return loss * self.get_loss_scale()

    def reload_model_params(self):
        for c in self.chunks:
            c.reload_master_from_params()

    def wait_param_sync(self):
        """Make the model parameters current (dist-opt all-gather in flight)."""
        for m in self.models:
            m.wait_param_sync()

    def _sp_norm_params(self):
        for m in self.models:
            for p in m.module.parameters():
                if getattr(p, "sequence_parallel", False):
                    yield p

    def allreduce_layernorm_grads(self, args):
        """SP: norm weights see only this rank's sequence shard -> sum over TP.

        Runs AFTER the DP grad sync has completed (``reduce_model_grads``): the
        DP collectives write the same grad buffer asynchronously, so touching
        it earlier would race with RCCL.  TP-sum and DP-average commute."""
        if state.get_tensor_model_parallel_world_size() > 1 and args.sequence_parallel:
            grads = [p.main_grad for p in self._sp_norm_params()]
            if grads:
                flat = torch._utils._flatten_dense_tensors(grads)
                comm.all_reduce(flat, group=state.get_tensor_model_parallel_group())
                for g, s in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
                    g.copy_(s)

    def _unwrapped(self, idx):
        from ..utils.misc import unwrap_model
        return unwrap_model(self.models[idx])

    def allreduce_word_embedding_grads(self, args):
        """Tied embeddings with PP > 1: sum word-embedding grads of first+last stage
        (reference ``optimizer.py:203-229``).  Runs BEFORE the DP reduction of the
        held embedding bucket, for the plain and the distributed optimizer alike."""
        if not (state.is_rank_in_embedding_group(ignore_virtual=True)
                and state.get_pipeline_model_parallel_world_size() > 1):
            return
        if state.is_pipeline_first_stage(ignore_virtual=True):
            idx = 0
        elif state.is_pipeline_last_stage(ignore_virtual=True):
            idx = len(self.models) - 1
        else:
            idx = 0
        unwrapped = self._unwrapped(idx)
        if getattr(unwrapped, "share_word_embeddings", False):
            w = unwrapped.word_embeddings_weight()
            self.models[idx]._zero_untouched([w])
            comm.all_reduce(w.main_grad, group=state.get_embedding_group())

    def allreduce_position_embedding_grads(self, args):
        """T5 with a PP split rank: encoder and decoder first stages share the
        position embeddings (reference ``optimizer.py:232-248``)."""
        if state.is_rank_in_position_embedding_group() and \
                state.get_pipeline_model_parallel_world_size() > 1 and \
                args.pipeline_model_parallel_split_rank is not None:
            unwrapped = self._unwrapped(0)
            pe = unwrapped.language_model.embedding.position_embeddings.weight
            self.models[0]._zero_untouched([pe])
            comm.all_reduce(pe.main_grad, group=state.get_position_embedding_group())

    def allreduce_embedding_grads(self, args):
        self.allreduce_word_embedding_grads(args)
        self.allreduce_position_embedding_grads(args)

    def reduce_model_grads(self, args, timers):
        """Order: (1) cross-stage embedding sums on the still-held, complete
        embedding grads; (2) launch the held buckets and wait for every DP
        bucket; (3) SP layer-norm TP sums on the now quiescent buffer."""
        timers("embedding-grads-all-reduce", log_level=1).start(barrier=args.barrier_with_L1_time)
        self.allreduce_embedding_grads(args)
        timers("embedding-grads-all-reduce").stop()
        name = "grads-reduce-scatter" if self.use_distributed_optimizer else "grads-all-reduce"
        timers(name, log_level=1).start(barrier=args.barrier_with_L1_time)
        for m in self.models:
            m.finish_grad_sync()
        timers(name).stop()
        timers("layernorm-grads-all-reduce", log_level=1).start(barrier=args.barrier_with_L1_time)
        self.allreduce_layernorm_grads(args)
        timers("layernorm-grads-all-reduce").stop()

    def gather_model_params(self, args, timers):
        if not self.use_distributed_optimizer:
            return
        timers("params-all-gather", log_level=1).start(barrier=args.barrier_with_L1_time)
        for m in self.models:
            m.start_param_sync()
        timers("params-all-gather").stop()

    # -- norm / clip -----------------------------------------------------------
    def _norm_group(self):
        if self.use_distributed_optimizer:
            return None  # world (reference distrib_optimizer.py:408-413)
        return state.get_model_parallel_group()

    def _grad_norm_sq(self):
        tot = None
        for c in self.chunks:
            v = K.grad_norm_sq(c.ddp.grad_buffer, c.plan).reshape(1).float()
            tot = v if tot is None else tot + v
        tot = comm.fold_xgmi_error(tot)  # a timed-out xGMI wait skips the step everywhere
        if dist.is_initialized():
            comm.all_reduce(tot, group=self._norm_group())
        return tot

    def count_zeros(self):
        z = sum(K.count_zeros(c.ddp.grad_buffer, c.plan) for c in self.chunks)
        t = torch.tensor([float(z)], device=self.chunks[0].master.device)
        if dist.is_initialized():
            comm.all_reduce(t, group=self._norm_group())
        return int(t.item())

    # -- lazy step resolution ----------------------------------------------------
    def register_scheduler_step(self, scheduler, increment):
        """``train_step`` advanced ``scheduler`` by ``increment`` samples for the
        last step; undone if that step turns out to have been skipped."""
        if self._pending is not None:
            self._pending.sched = (scheduler, increment)

    def resolve_pending(self):
        """Settle the previous step: roll back the scheduler if it was skipped."""
        r = self._pending
        if r is None or r.resolved:
            return
        r.resolved = True
        skipped = r.found_inf
        self.found_inf = skipped
        if not skipped:
            self._host_step += 1
        if skipped and r.sched is not None:
            sched, inc = r.sched
            sched.rollback(inc)
        for g in self.param_groups:
            if "step" in g:
                g["step"] = self._host_step

    # -- step -------------------------------------------------------------------
    @torch.no_grad()
    def step(self, args, timers):
        self.resolve_pending()
        for m in self.models:
            m.wait_param_sync()
        timers("optimizer-unscale-and-check-inf", log_level=1).start(
            barrier=args.barrier_with_L1_time)
        inv_scale = self.grad_scaler.inv_scale if self.grad_scaler is not None else None
        norm_sq = self._grad_norm_sq()
        timers("optimizer-unscale-and-check-inf").stop()
        timers("optimizer-clip-main-grad", log_level=1).start(barrier=args.barrier_with_L1_time)
        K.step_prep(norm_sq, inv_scale, self.clip_grad, self._st)
        timers("optimizer-clip-main-grad").stop()
        if self.grad_scaler is not None:
            self.grad_scaler.update(self._st[1:2] != 0)
        num_zeros = self.count_zeros() if self.log_num_zeros_in_grad else None
        timers("optimizer-inner-step", log_level=1).start(barrier=args.barrier_with_L1_time)
        lrs = [g["lr"] for g in self.param_groups]
        wds = [g["weight_decay"] for g in self.param_groups]
        for c in self.chunks:
            if self.kind == "adam":
                K.adam_step(c.master, c.model_out, c.ddp.grad_buffer, c.exp_avg, c.exp_avg_sq,
                            c.plan, lrs, wds, self.beta1, self.beta2, self.eps,
                            self._host_step + 1, 1.0, dev_state=self._st)
            else:
                K.sgd_step(c.master, c.model_out, c.ddp.grad_buffer, c.momentum, c.plan, lrs,
                           wds, self.sgd_momentum, 1.0, dev_state=self._st)
        timers("optimizer-inner-step").stop()
        timers("optimizer-copy-main-to-model-params", log_level=1).start(
            barrier=args.barrier_with_L1_time)
        self.gather_model_params(args, timers)
        timers("optimizer-copy-main-to-model-params").stop()
        # parameters were rewritten through the flat buffers (not through the
        # Parameter objects, whose _version does not move): invalidate the
        # derived copies keyed on the weight generation (decode-packed weights)
        decode_pack.bump_weight_generation()
        res = StepResult(self._st)
        self._pending = res
        return res, LazyScalar(lambda: (None if res.found_inf else res.grad_norm)), num_zeros

    # -- checkpoint state ---------------------------------------------------------
    def _param_order(self):
        order = []
        for g in self.param_groups:
            order.extend(g["params"])
        return order

    def _chunk_of(self, p):
        for c in self.chunks:
            if p in c.ddp.param_index:
                return c
        raise KeyError("param not managed by this optimizer")

    def _full_param_state(self, flat_attr, p):
        """Full (unsharded) fp32 state of ``p`` (non-distributed optimizer only)."""
        c = self._chunk_of(p)
        out = torch.empty(p.numel(), dtype=torch.float32, device=c.master.device)
        c.read_param_range(getattr(c, flat_attr), p, 0, p.numel(), out)
        return out.view_as(p)

    def _group_meta(self, g):
        return {k: v for k, v in g.items() if k != "params"}

    def state_dict(self):
        self.resolve_pending()
        if self.use_distributed_optimizer:
            return self._dist_state_dict()
        order = self._param_order()
        st = {}
        for i, p in enumerate(order):
            st[i] = {k: self._full_param_state(_attr_of(k), p) for k in self._state_keys()}
        groups, idx = [], 0
        for g in self.param_groups:
            d = self._group_meta(g)
            d["params"] = list(range(idx, idx + len(g["params"])))
            idx += len(g["params"])
            groups.append(d)
        sd = {"optimizer": {"state": st, "param_groups": groups}}
        if self.grad_scaler is not None:
            sd["grad_scaler"] = self.grad_scaler.state_dict()
        if any(c.model_out is not None for c in self.chunks):
            sd["fp32_from_fp16_params"] = [[self._full_param_state("master", p)
                                            for p in g["params"]] for g in self.param_groups]
        return sd

    def _state_keys(self):
        return ("exp_avg", "exp_avg_sq") if self.kind == "adam" else ("momentum_buffer",)

    def load_state_dict(self, sd, dp_peer_loader=None):
        """``dp_peer_loader(r)`` returns the distributed-optimizer state dict
        saved by DP rank ``r`` of this (TP, PP) rank (needed with the distributed
        optimizer: shards are cut by the reference layout, not ours)."""
        if self.use_distributed_optimizer or "shard_fp32_from_float16_groups" in sd:
            return self._dist_load_state_dict(sd, dp_peer_loader)
        opt = sd["optimizer"]
        order = self._param_order()
        for i, p in enumerate(order):
            s = opt["state"].get(i, opt["state"].get(str(i)))
            if s is None:
                continue
            c = self._chunk_of(p)
            for k in self._state_keys():
                if k in s:
                    c.write_param_range(getattr(c, _attr_of(k)), p, 0,
                                        s[k].reshape(-1).to(c.master.device, torch.float32))
        self._restore_groups(opt["param_groups"])
        if "grad_scaler" in sd and self.grad_scaler is not None and sd["grad_scaler"]:
            self.grad_scaler.load_state_dict(sd["grad_scaler"])
        if "fp32_from_fp16_params" in sd:
            for g, saved in zip(self.param_groups, sd["fp32_from_fp16_params"]):
                for p, t in zip(g["params"], saved):
                    c = self._chunk_of(p)
                    c.write_param_range(c.master, p, 0,
                                        t.reshape(-1).to(c.master.device, torch.float32))
            self._push_master_to_model()

    def _push_master_to_model(self):
        decode_pack.bump_weight_generation()
        for c in self.chunks:
            if c.model_out is not None:
                K.copy_master_to_model(c.master, c.model_out, c.plan)
        if self.use_distributed_optimizer:
            for m in self.models:
                m.all_gather_params()

    def _restore_groups(self, groups):
        step = 0
        for g, s in zip(self.param_groups, groups):
            for k in ("lr", "weight_decay"):
                if k in s:
                    g[k] = s[k]
        for s in groups:
            step = max(step, int(s.get("step", 0)))
        self._set_step(step)

    def _set_step(self, step):
        self._host_step = step
        self._st[2] = float(step)
        for g in self.param_groups:
            if "step" in g:
                g["step"] = step

    # -- distributed-optimizer state in the reference layout ---------------------
    def _ref_plan(self, dp, r):
        """Reference shard plan of DP rank ``r`` at DP size ``dp``: squeezed groups
        of [(chunk_index, param, lo, hi)] in the order the reference's
        ``build_optimizer_group_ranges`` lists them."""
        groups = [[] for _ in self.param_groups]
        for ci, c in enumerate(self.chunks):
            params = [p for p in c.ddp.module.parameters() if p.requires_grad]
            total = sum(p.numel() for p in params)
            size = int(math.ceil(total / dp))
            r_lo, r_hi = r * size, min(total, (r + 1) * size)
            end = total
            for p in params:  # forward order; packed from the buffer end
                start = end - p.numel()
                a, b = max(start, r_lo), min(end, r_hi)
                if a < b:
                    groups[self._group_of_param[p]].append((ci, p, a - start, b - start))
                end = start
        kept = [(gi, g) for gi, g in enumerate(groups) if g]
        return kept

    def _dist_state_dict(self):
        dp = state.get_data_parallel_world_size()
        r = state.get_data_parallel_rank()
        plan = self._ref_plan(dp, r)
        wanted = {}
        for _, entries in plan:
            for ci, p, lo, hi in entries:
                wanted[p] = (ci, lo, hi)
        keys = ["master"] + list(self._state_keys())
        shards = {p: {} for p in wanted}
        # bucket by bucket (every rank walks all buckets: the gathers are collective)
        for ci, c in enumerate(self.chunks):
            for b in c.ddp.buckets:
                for k in keys:
                    flat = c.master if k == "master" else getattr(c, _attr_of(k))
                    m_off, _, n = c.ranges[b.index]
                    full = torch.empty(b.numel, dtype=torch.float32, device=flat.device)
                    comm.all_gather_into(full, flat[m_off:m_off + n], group=c.ddp.dp_group)
                    for p in b.params:
                        if p in wanted and wanted[p][0] == ci:
                            _, lo, hi = wanted[p]
                            off, _ = c.ddp.param_index[p]
                            s = off - b.start
                            shards[p][k] = full[s + lo:s + hi].clone()
        st, groups, fp32_groups, idx = {}, [], [], 0
        for gi, entries in plan:
            d = self._group_meta(self.param_groups[gi])
            d["params"] = list(range(idx, idx + len(entries)))
            groups.append(d)
            fg = []
            for ci, p, lo, hi in entries:
                st[idx] = {k: shards[p][k] for k in self._state_keys()}
                fg.append(shards[p]["master"])
                idx += 1
            fp32_groups.append(fg if self.chunks[0].half_params else [])
        sd = {"optimizer": {"state": st, "param_groups": groups},
              "shard_fp32_from_float16_groups": fp32_groups,
              # MI355X addition (ignored by the reference loader): what the shard
              # layout depends on, so a load can verify / reshard.
              "layout": {"format": "megatron-distrib-optimizer-v1", "dp_size": dp,
                         "dp_rank": r,
                         "chunk_numel": [sum(p.numel() for p in c.ddp.module.parameters()
                                             if p.requires_grad) for c in self.chunks]}}
        if self.grad_scaler is not None:
            sd["grad_scaler"] = self.grad_scaler.state_dict()
        return sd

    def _dist_load_state_dict(self, sd, dp_peer_loader):
        layout = sd.get("layout", {})
        numels = [sum(p.numel() for p in c.ddp.module.parameters() if p.requires_grad)
                  for c in self.chunks]
        if layout.get("chunk_numel") is not None and list(layout["chunk_numel"]) != numels:
            raise RuntimeError(
                f"distributed-optimizer checkpoint was written for a model with "
                f"{layout['chunk_numel']} parameters per chunk, this model has {numels}")
        saved_dp = layout.get("dp_size")
        if saved_dp is None:
            saved_dp = dp_peer_loader.num_ranks() if dp_peer_loader is not None \
                else state.get_data_parallel_world_size()
        my_dp = state.get_data_parallel_world_size()
        if dp_peer_loader is None and (saved_dp != 1 or my_dp != 1) and \
                not (saved_dp == my_dp and not self.use_distributed_optimizer):
            raise RuntimeError("loading distributed-optimizer state needs the DP peer files")
        keys = ["master"] + list(self._state_keys())
        for r in range(saved_dp):
            src = sd if (dp_peer_loader is None or r == layout.get("dp_rank", -1)) \
                else dp_peer_loader(r)
            plan = self._ref_plan(saved_dp, r)
            if len(src["optimizer"]["param_groups"]) != len(plan):
                raise RuntimeError(f"distributed-optimizer shard {r}: group count mismatch "
                                   f"({len(src['optimizer']['param_groups'])} vs {len(plan)})")
            idx = 0
            for gpos, (gi, entries) in enumerate(plan):
                masters = src["shard_fp32_from_float16_groups"][gpos] \
                    if src.get("shard_fp32_from_float16_groups") else []
                for j, (ci, p, lo, hi) in enumerate(entries):
                    c = self.chunks[ci]
                    s = src["optimizer"]["state"].get(idx, src["optimizer"]["state"].get(str(idx)))
                    for k in keys:
                        if k == "master":
                            if not masters:
                                continue
                            t = masters[j]
                            flat = c.master
                        else:
                            if s is None or k not in s:
                                continue
                            t = s[k]
                            flat = getattr(c, _attr_of(k))
                        t = t.reshape(-1)
                        if t.numel() != hi - lo:
                            raise RuntimeError(f"distributed-optimizer shard {r}: param "
                                               f"{idx} has {t.numel()} elements, expected "
                                               f"{hi - lo}")
                        c.write_param_range(flat, p, lo, t.to(flat.device, torch.float32))
                    idx += 1
            if r == 0 or src is sd:
                step = max([int(g.get("step", 0)) for g in src["optimizer"]["param_groups"]]
                           + [0])
                self._set_step(step)
        if self.grad_scaler is not None and sd.get("grad_scaler"):
            self.grad_scaler.load_state_dict(sd["grad_scaler"])
        if self.chunks[0].half_params:
            self._push_master_to_model()


def _attr_of(key):
    return {"exp_avg": "exp_avg", "exp_avg_sq": "exp_avg_sq",
            "momentum_buffer": "momentum", "master": "master"}[key]

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
"""
import math

import torch
import torch.distributed as dist

from ..parallel import state
from ..parallel.tensor.layers import param_is_not_tensor_parallel_duplicate
from ..models.module import param_is_not_shared
from ..ops import optim_kernels as K


class _ChunkState:
    """Flat optimizer state for one DDP model chunk."""

    def __init__(self, ddp, group_of_param, master_from_params, kind):
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
        if kind == "adam":
            self.exp_avg = torch.zeros(self.numel, dtype=torch.float32, device=device)
            self.exp_avg_sq = torch.zeros(self.numel, dtype=torch.float32, device=device)
        else:
            self.momentum = torch.zeros(self.numel, dtype=torch.float32, device=device)
        # segments: intersection of each param's [off, off+n) with the owned ranges
        segs = []
        self.param_master_ranges = {}
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
                  "betas": (adam_beta1, adam_beta2), "eps": adam_eps, "bias_correction": True,
                  "amsgrad": False, "step": 0}
            self.param_groups.append(pg)
            for p in pg["params"]:
                group_of_param[p] = gi
        self.chunks = [_ChunkState(m, group_of_param, True, kind) for m in models]
        self._step = 0
        self.found_inf = False

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

    def _sp_norm_params(self):
        for m in self.models:
            for p in m.module.parameters():
                if getattr(p, "sequence_parallel", False):
                    yield p

    def allreduce_layernorm_grads(self, args):
        """SP: norm weights see only this rank's sequence shard -> sum over TP."""
        if state.get_tensor_model_parallel_world_size() > 1 and args.sequence_parallel:
            grads = [p.main_grad for p in self._sp_norm_params()]
            if grads:
                flat = torch._utils._flatten_dense_tensors(grads)
                dist.all_reduce(flat, group=state.get_tensor_model_parallel_group())
                for g, s in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
                    g.copy_(s)

    def allreduce_embedding_grads(self, args):
        """Tied embeddings with PP > 1: sum word-embedding grads of first+last stage."""
        if not (state.is_rank_in_embedding_group(ignore_virtual=True)
                and state.get_pipeline_model_parallel_world_size() > 1):
            return
        from ..utils.misc import unwrap_model
        if state.is_pipeline_first_stage(ignore_virtual=True):
            unwrapped = unwrap_model(self.models[0])
        elif state.is_pipeline_last_stage(ignore_virtual=True):
            unwrapped = unwrap_model(self.models[-1])
        else:
            return
        if getattr(unwrapped, "share_word_embeddings", False):
            w = unwrapped.word_embeddings_weight()
            dist.all_reduce(w.main_grad, group=state.get_embedding_group())

    def reduce_model_grads(self, args, timers):
        timers("layernorm-grads-all-reduce", log_level=1).start(barrier=args.barrier_with_L1_time)
        self.allreduce_layernorm_grads(args)
        timers("layernorm-grads-all-reduce").stop()
        name = "grads-reduce-scatter" if self.use_distributed_optimizer else "grads-all-reduce"
        timers(name, log_level=1).start(barrier=args.barrier_with_L1_time)
        for m in self.models:
            m.finish_grad_sync()
        timers(name).stop()
        timers("embedding-grads-all-reduce", log_level=1).start(barrier=args.barrier_with_L1_time)
        self.allreduce_embedding_grads(args)
        timers("embedding-grads-all-reduce").stop()

    def gather_model_params(self, args, timers):
        if not self.use_distributed_optimizer:
            return
        timers("params-all-gather", log_level=1).start(barrier=args.barrier_with_L1_time)
        for m in self.models:
            m.all_gather_params()
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
        if dist.is_initialized():
            dist.all_reduce(tot, group=self._norm_group())
        return tot

    def count_zeros(self):
        z = sum(K.count_zeros(c.ddp.grad_buffer, c.plan) for c in self.chunks)
        t = torch.tensor([float(z)], device=self.chunks[0].master.device)
        if dist.is_initialized():
            dist.all_reduce(t, group=self._norm_group())
        return int(t.item())

    # -- step -------------------------------------------------------------------
    @torch.no_grad()
    def step(self, args, timers):
        timers("optimizer-unscale-and-check-inf", log_level=1).start(
            barrier=args.barrier_with_L1_time)
        inv_scale = 1.0
        if self.grad_scaler is not None:
            inv_scale = float(self.grad_scaler.inv_scale.item())
        norm_sq = self._grad_norm_sq()
        timers("optimizer-unscale-and-check-inf").stop()
        timers("optimizer-clip-main-grad", log_level=1).start(barrier=args.barrier_with_L1_time)
        raw = float(norm_sq.item())
        grad_norm = math.sqrt(raw) * inv_scale if math.isfinite(raw) else float("nan")
        timers("optimizer-clip-main-grad").stop()
        found_inf = not math.isfinite(raw)
        if self.grad_scaler is not None:
            self.grad_scaler.update(found_inf)
        if found_inf:
            # fp16 overflow or (EPFL addition) non-finite norm: skip the step.
            self.found_inf = True
            return False, None, None
        self.found_inf = False
        coef = 1.0
        if self.clip_grad > 0.0:
            c = self.clip_grad / (grad_norm + 1.0e-6)
            if c < 1.0:
                coef = c
        num_zeros = self.count_zeros() if self.log_num_zeros_in_grad else None
        timers("optimizer-inner-step", log_level=1).start(barrier=args.barrier_with_L1_time)
        self._step += 1
        for g in self.param_groups:
            g["step"] = self._step
        lrs = [g["lr"] for g in self.param_groups]
        wds = [g["weight_decay"] for g in self.param_groups]
        scale = coef * inv_scale
        for c in self.chunks:
            if self.kind == "adam":
                K.adam_step(c.master, c.model_out, c.ddp.grad_buffer, c.exp_avg, c.exp_avg_sq,
                            c.plan, lrs, wds, self.beta1, self.beta2, self.eps, self._step, scale)
            else:
                K.sgd_step(c.master, c.model_out, c.ddp.grad_buffer, c.momentum, c.plan, lrs,
                           wds, self.sgd_momentum, scale)
        timers("optimizer-inner-step").stop()
        timers("optimizer-copy-main-to-model-params", log_level=1).start(
            barrier=args.barrier_with_L1_time)
        self.gather_model_params(args, timers)
        timers("optimizer-copy-main-to-model-params").stop()
        return True, grad_norm, num_zeros

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

    def _param_views(self, flat_attr, p):
        c = self._chunk_of(p)
        ranges = c.param_master_ranges.get(p, [])
        flat = getattr(c, flat_attr)
        if len(ranges) == 1 and ranges[0][1] == 0 and ranges[0][2] == p.numel():
            return flat[ranges[0][0]:ranges[0][0] + p.numel()].view_as(p)
        return None

    def state_dict(self):
        """apex-FusedAdam-compatible layout when unsharded; flat shards otherwise."""
        if self.use_distributed_optimizer:
            return {"flat_shards": [{"master": c.master,
                                     **({"exp_avg": c.exp_avg, "exp_avg_sq": c.exp_avg_sq}
                                        if self.kind == "adam" else {"momentum": c.momentum})}
                                    for c in self.chunks],
                    "param_groups": [{k: v for k, v in g.items() if k != "params"}
                                     for g in self.param_groups],
                    "grad_scaler": self.grad_scaler.state_dict() if self.grad_scaler else None,
                    "step": self._step}
        order = self._param_order()
        st = {}
        if self.kind == "adam":
            for i, p in enumerate(order):
                st[i] = {"exp_avg": self._param_views("exp_avg", p),
                         "exp_avg_sq": self._param_views("exp_avg_sq", p)}
        else:
            for i, p in enumerate(order):
                st[i] = {"momentum_buffer": self._param_views("momentum", p)}
        groups, idx = [], 0
        for g in self.param_groups:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = list(range(idx, idx + len(g["params"])))
            idx += len(g["params"])
            groups.append(d)
        sd = {"optimizer": {"state": st, "param_groups": groups}}
        if self.grad_scaler is not None:
            sd["grad_scaler"] = self.grad_scaler.state_dict()
        if any(c.model_out is not None for c in self.chunks):
            sd["fp32_from_fp16_params"] = [[self._param_views("master", p) for p in g["params"]]
                                           for g in self.param_groups]
        return sd

    def load_state_dict(self, sd):
        if "flat_shards" in sd:
            for c, src in zip(self.chunks, sd["flat_shards"]):
                c.master.copy_(src["master"])
                if self.kind == "adam":
                    c.exp_avg.copy_(src["exp_avg"])
                    c.exp_avg_sq.copy_(src["exp_avg_sq"])
                else:
                    c.momentum.copy_(src["momentum"])
            self._step = sd.get("step", 0)
            if self.grad_scaler is not None and sd.get("grad_scaler"):
                self.grad_scaler.load_state_dict(sd["grad_scaler"])
            self._restore_groups(sd["param_groups"])
            for c in self.chunks:
                if c.model_out is not None:
                    K.copy_master_to_model(c.master, c.model_out, c.plan)
            return
        opt = sd["optimizer"]
        order = self._param_order()
        for i, p in enumerate(order):
            s = opt["state"].get(i, opt["state"].get(str(i)))
            if s is None:
                continue
            if self.kind == "adam":
                self._param_views("exp_avg", p).copy_(s["exp_avg"])
                self._param_views("exp_avg_sq", p).copy_(s["exp_avg_sq"])
            elif "momentum_buffer" in s:
                self._param_views("momentum", p).copy_(s["momentum_buffer"])
        self._restore_groups(opt["param_groups"])
        if "grad_scaler" in sd and self.grad_scaler is not None:
            self.grad_scaler.load_state_dict(sd["grad_scaler"])
        if "fp32_from_fp16_params" in sd:
            for g, saved in zip(self.param_groups, sd["fp32_from_fp16_params"]):
                for p, t in zip(g["params"], saved):
                    self._param_views("master", p).copy_(t)
            for c in self.chunks:
                if c.model_out is not None:
                    K.copy_master_to_model(c.master, c.model_out, c.plan)

    def _restore_groups(self, groups):
        for g, s in zip(self.param_groups, groups):
            for k in ("lr", "weight_decay", "step"):
                if k in s:
                    g[k] = s[k]
        self._step = max([g.get("step", 0) for g in self.param_groups] + [self._step])

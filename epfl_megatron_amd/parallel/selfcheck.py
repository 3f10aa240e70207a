"""Startup self-check of the collective semantics the framework relies on.

The CPU tests exercise every collective path on ``gloo``; the first run that
can disagree with them is the first multi-GPU RCCL run.  So right after the
process groups exist, every rank runs a handful of tiny collectives on the
REAL backend and compares the results with values it can compute locally:

* DP group(s) (every ``--ddp_comm_groups`` communicator) and TP group:
  - in-place ``reduce_scatter_tensor`` with ``ReduceOp.AVG`` on fp32 (the DDP
    bucket path, ``parallel/ddp.py``), sync and async;
  - in-place ``all_gather_into_tensor`` on bf16 and fp32 (dist-opt parameter
    gather, SP all-gather), async;
  - ``all_reduce`` SUM on fp32 and MAX on fp32 (grad norm / inf checks);
* PP group: one batched send/recv between every pair of adjacent stages
  through ``comm.p2p`` (the pipeline schedules' path).

Any mismatch raises ``RuntimeError`` naming the group and the operation
before any model memory is allocated.  Cost: ~20 collectives of <= 1 KiB.
Reference: the reference had no such check (``megatron/initialize.py:124-159``).

Environment knobs.  ``EMA_*`` variables are read at import time, and several
change how many collectives a step posts, or their shapes (``EMA_SP_CHUNKS``,
``EMA_SP_MLP_PIECES``, ``EMA_FUSED_MLP``, ``EMA_NT_GEMM``, ``EMA_COMM_CHECK``,
...).  A rank started with a different value would post a different sequence
and hang RCCL mid-step, so :func:`check_env_agrees` all-gathers a hash of every
``EMA_*`` variable that is not known to be rank-local (kernel tuning, tracing)
and refuses to start on a mismatch, naming the differing variables.
"""
import hashlib
import json
import os

import torch
import torch.distributed as dist

from . import comm, state

# EMA_* variables that only tune a kernel's schedule or a rank-local aid; they
# may differ between ranks.  Every other EMA_* variable is treated as able to
# change the collective sequence (conservative: a new knob is checked unless
# it is listed here).
_LOCAL_KNOBS = ("EMA_TRACE", "EMA_STRICT_KERNELS", "EMA_OFFLOAD_ARCH", "EMA_EMBEDDED",
                "EMA_XGMI_TIMEOUT_MS", "EMA_LOOPBACK_STREAM", "EMA_DGRAD_WT",
                "EMA_NORM_MAIN_GRAD", "EMA_SKINNY_PACK", "EMA_SKINNY_WAVES",
                "EMA_SKINNY_PERSIST", "EMA_WGRAD_MIN_TILES", "EMA_LOOPBACK_KEPT_POOL")
_LOCAL_PREFIXES = ("EMA_GEMM_", "EMA_WGRAD_", "EMA_FA_", "EMA_RMS_")


def structural_env(environ=None):
    """The ``EMA_*`` variables that must agree across ranks (sorted dict)."""
    environ = os.environ if environ is None else environ
    return {k: environ[k] for k in sorted(environ)
            if k.startswith("EMA_") and k not in _LOCAL_KNOBS
            and not k.startswith(_LOCAL_PREFIXES)}


def check_env_agrees(environ=None):
    """All-gather a hash of :func:`structural_env` over the world; raise
    ``RuntimeError`` naming the variables whose values differ.  Returns the
    number of ranks compared (1: nothing to do)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return 1
    env = structural_env(environ)
    digest = hashlib.sha256(json.dumps(env, sort_keys=True).encode()).digest()
    mine = torch.tensor([int.from_bytes(digest[:7], "little")], dtype=torch.int64, device=_dev())
    world = dist.get_world_size()
    every = torch.empty(world, dtype=torch.int64, device=_dev())
    comm.all_gather_into(every, mine)
    if bool((every == every[0]).all()):
        return world
    envs = [None] * world  # the slow path names the culprits (host objects)
    dist.all_gather_object(envs, env)
    keys = sorted(set().union(*envs))
    diff = {k: [e.get(k) for e in envs] for k in keys if len({e.get(k) for e in envs}) > 1}
    raise RuntimeError(
        "EMA_* environment differs between ranks; these variables change the collective "
        "sequence and must be identical on every rank (value per rank, None = unset): "
        + "; ".join(f"{k}={v}" for k, v in diff.items()))


def _dev():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")


def _fail(what, got, want):
    raise RuntimeError(
        f"collective self-check failed: {what}\n  got  {got.tolist()}\n  want {want.tolist()}\n"
        "The backend does not implement this collective as the framework assumes "
        "(see epfl_megatron_amd/parallel/selfcheck.py).")


def _check_group(name, group, size, rank, dev, n=8):
    if size <= 1:
        return 0
    ks = torch.arange(size, dtype=torch.float64)
    # 1. in-place reduce-scatter, AVG, fp32: rank k contributes k + 2 j at j
    for async_op in (False, True):
        buf = (rank + 2 * torch.arange(size * n, dtype=torch.float64)).to(torch.float32).to(dev)
        out = buf[rank * n:(rank + 1) * n]
        h = comm.reduce_scatter_into(out, buf, group=group, async_op=async_op, op="avg")
        if h is not None:
            h.wait()
        j = torch.arange(rank * n, (rank + 1) * n, dtype=torch.float64)
        want = (ks.mean() + 2 * j).to(torch.float32)
        if not torch.allclose(out.cpu(), want, rtol=0, atol=1e-5):
            _fail(f"{name}: in-place reduce_scatter(AVG, fp32, async={async_op})", out.cpu(), want)
    # 2. in-place all-gather, bf16 and fp32: chunk k = 10 k + i (exact in bf16)
    for dt in (torch.bfloat16, torch.float32):
        buf = torch.zeros(size * n, dtype=dt, device=dev)
        buf[rank * n:(rank + 1) * n] = (10 * rank + torch.arange(n)).to(dt).to(dev)
        h = comm.all_gather_into(buf, buf[rank * n:(rank + 1) * n], group=group, async_op=True)
        h.wait()
        want = (10 * torch.arange(size).repeat_interleave(n) + torch.arange(n).repeat(size)).to(dt)
        if not torch.equal(buf.cpu(), want):
            _fail(f"{name}: in-place all_gather({dt})", buf.cpu(), want)
    # 3. all-reduce SUM and MAX, fp32
    t = torch.full((4,), float(rank + 1), dtype=torch.float32, device=dev)
    comm.all_reduce(t, group=group)
    want = torch.full((4,), float(size * (size + 1) // 2), dtype=torch.float32)
    if not torch.equal(t.cpu(), want):
        _fail(f"{name}: all_reduce(SUM, fp32)", t.cpu(), want)
    t = torch.full((4,), float(rank), dtype=torch.float32, device=dev)
    comm.all_reduce(t, group=group, op="max")
    want = torch.full((4,), float(size - 1), dtype=torch.float32)
    if not torch.equal(t.cpu(), want):
        _fail(f"{name}: all_reduce(MAX, fp32)", t.cpu(), want)
    return 6


def _check_pipeline(dev):
    pp = state.get_pipeline_model_parallel_world_size()
    if pp <= 1:
        return 0
    import torch.distributed as dist
    group = state.get_pipeline_model_parallel_group()
    me = dist.get_rank()
    ops, recv = [], None
    if not state.is_pipeline_last_stage(ignore_virtual=True):
        ops.append(("send", torch.full((4,), float(me), device=dev),
                    state.get_pipeline_model_parallel_next_rank()))
    if not state.is_pipeline_first_stage(ignore_virtual=True):
        recv = torch.empty(4, device=dev)
        ops.append(("recv", recv, state.get_pipeline_model_parallel_prev_rank()))
    comm.p2p(ops, group=group)
    if recv is not None:
        want = torch.full((4,), float(state.get_pipeline_model_parallel_prev_rank()))
        if not torch.equal(recv.cpu(), want):
            _fail("pp: send/recv between adjacent stages", recv.cpu(), want)
    return 1


def collective_selfcheck(verbose=True):
    """Run the checks on every group this rank belongs to; returns the count."""
    dev = _dev()
    n = 1 if check_env_agrees() > 1 else 0
    dp_groups = state.get_data_parallel_comm_groups()
    for i, g in enumerate(dp_groups):
        n += _check_group(f"dp[{i}]", g, state.get_data_parallel_world_size(),
                          state.get_data_parallel_rank(), dev)
    n += _check_group("tp", state.get_tensor_model_parallel_group(),
                      state.get_tensor_model_parallel_world_size(),
                      state.get_tensor_model_parallel_rank(), dev)
    if state.get_context_parallel_group() is not None:
        n += _check_group("cp", state.get_context_parallel_group(),
                          state.get_context_parallel_world_size(),
                          state.get_context_parallel_rank(), dev)
    n += _check_pipeline(dev)
    comm.report(reset=True)  # keep the check out of the training accounting
    if verbose:
        import torch.distributed as dist
        if dist.get_rank() == 0:
            print(f"> collective self-check passed ({n} checks; dp={state.get_data_parallel_world_size()}"
                  f" x{len(dp_groups)} comm groups, tp={state.get_tensor_model_parallel_world_size()}, "
                  f"pp={state.get_pipeline_model_parallel_world_size()}, "
                  f"cp={state.get_context_parallel_world_size()})", flush=True)
    return n

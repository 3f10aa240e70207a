"""Sharded checkpoint save/load (format: SURVEY Appendix B, reference
``megatron/checkpointing.py``).

Layout::

    <dir>/latest_checkpointed_iteration.txt            "<iteration>" | "release"
    <dir>/iter_XXXXXXX|release/mp_rank_TT[_PPP]/model_optim_rng.pt
    with --use_distributed_optimizer:
        mp_rank_TT[_PPP]/model_rng.pt + mp_rank_TT[_PPP]_DDD/optim.pt

Top-level keys: ``args`` (Namespace), ``checkpoint_version`` 3.0,
``iteration``, ``model`` (``model0..`` for virtual PP), ``rng_state``,
``optimizer``, ``opt_param_scheduler``.

Loading never executes code from the file: ``torch.load(weights_only=True)``
with an allow-list (Namespace, torch dtypes, our enums — also under the
reference's ``megatron.model.enums`` names so reference-written checkpoints
load).  ``--async_save`` stages tensors to pinned host memory and writes on a
background thread (MI355X addition; the reference writes synchronously).
"""
import argparse
import os
import random
import sys
import threading

import numpy as np
import torch
import torch.distributed as dist

from . import ckpt_pickle, global_vars
from .ops import decode_pack
from .parallel import state
from .parallel.tensor.random import get_cuda_rng_tracker
from .models import enums as _enums
from .utils.misc import print_rank_0, unwrap_model

_CHECKPOINT_VERSION = None
_ASYNC_THREAD = None


def set_checkpoint_version(value):
    global _CHECKPOINT_VERSION
    if _CHECKPOINT_VERSION is not None and _CHECKPOINT_VERSION != value:
        raise AssertionError("checkpoint versions do not match")
    _CHECKPOINT_VERSION = value


def get_checkpoint_version():
    return _CHECKPOINT_VERSION


def _safe_globals():
    allow = [argparse.Namespace]
    for e in _enums.ALL_ENUMS:
        allow.append(e)
        allow.append((e, f"megatron.model.enums.{e.__name__}"))
    # very old checkpoints pickled their loss scaler objects (reference
    # checkpointing.py:457-468 remaps these module paths)
    from .fp16_deprecated import loss_scaler as _ls
    for cls in (_ls.LossScaler, _ls.DynamicLossScaler):
        allow.append(cls)
        for mod in ("fp16.loss_scaler", "megatron.fp16.loss_scaler",
                    "megatron.fp16_deprecated.loss_scaler"):
            allow.append((cls, f"{mod}.{cls.__name__}"))
    try:
        import numpy.core.multiarray as ma
        allow += [ma._reconstruct, np.ndarray, np.dtype, type(np.dtype(np.uint32))]
    except Exception:  # pragma: no cover
        pass
    return allow


def safe_load(path, map_location="cpu", mmap=False):
    """``torch.load(weights_only=True)`` with our allow-list."""
    with torch.serialization.safe_globals(_safe_globals()):
        return torch.load(path, map_location=map_location, weights_only=True, mmap=mmap)


class DPPeerLoader:
    """Reads the distributed-optimizer ``optim.pt`` of any DP rank of this
    (TP, PP) rank (``mp_rank_TT[_PPP]_RRR/optim.pt``, reference
    ``checkpointing.py:107-140``).  The optimizer state there is sharded by the
    reference buffer layout, so a rank gathers its own ranges from all of them
    — which also makes a load at a different DP size or bucket size work."""

    def __init__(self, load_dir, iteration, release):
        self.load_dir, self.iteration, self.release = load_dir, iteration, release
        model_name, _ = get_checkpoint_names(load_dir, iteration, True, release)
        self.prefix = os.path.dirname(model_name)

    def path(self, r):
        return self.prefix + f"_{r:03d}/optim.pt"

    def num_ranks(self):
        n = 0
        while os.path.exists(self.path(n)):
            n += 1
        return n

    def __call__(self, r):
        return safe_load(self.path(r), mmap=True)["optimizer"]


def check_checkpoint_args(checkpoint_args):
    args = global_vars.get_args()

    def _cmp(name, old_name=None):
        ck = getattr(checkpoint_args, old_name or name, None)
        if ck is None:
            return
        cur = getattr(args, name)
        if cur != ck:
            raise AssertionError(f"{name} value from checkpoint ({ck}) is not equal to the "
                                 f"input argument value ({cur}).")

    for n in ("num_layers", "hidden_size", "num_attention_heads"):
        _cmp(n)
    if getattr(checkpoint_args, "add_position_embedding", None) is not None and \
            args.position_embedding_type == _enums.PositionEmbeddingType.absolute:
        pass
    if get_checkpoint_version() and get_checkpoint_version() < 3.0:
        _cmp("tensor_model_parallel_size", "model_parallel_size")
    else:
        _cmp("tensor_model_parallel_size")
        _cmp("pipeline_model_parallel_size")


def ensure_directory_exists(filename):
    d = os.path.dirname(filename)
    if d:
        os.makedirs(d, exist_ok=True)


def get_checkpoint_names(checkpoints_path, iteration, use_distributed_optimizer, release=False,
                         pipeline_parallel=None, tensor_rank=None, pipeline_rank=None):
    directory = "release" if release else f"iter_{iteration:07d}"
    if pipeline_parallel is None:
        pipeline_parallel = state.get_pipeline_model_parallel_world_size() > 1
    if tensor_rank is None:
        tensor_rank = state.get_tensor_model_parallel_rank()
    if pipeline_rank is None:
        pipeline_rank = state.get_pipeline_model_parallel_rank()
    common = os.path.join(checkpoints_path, directory,
                          f"mp_rank_{tensor_rank:02d}" if not pipeline_parallel
                          else f"mp_rank_{tensor_rank:02d}_{pipeline_rank:03d}")
    if use_distributed_optimizer:
        model_name = os.path.join(common, "model_rng.pt")
        optim_name = os.path.join(common + f"_{state.get_data_parallel_rank():03d}", "optim.pt")
    else:
        model_name = optim_name = os.path.join(common, "model_optim_rng.pt")
    return model_name, optim_name


def get_checkpoint_tracker_filename(checkpoints_path):
    return os.path.join(checkpoints_path, "latest_checkpointed_iteration.txt")


def read_metadata(tracker_filename):
    with open(tracker_filename) as f:
        meta = f.read().strip()
    release = meta == "release"
    iteration = 0
    if not release:
        try:
            iteration = int(meta)
        except ValueError:
            print_rank_0(f"ERROR: Invalid metadata file {tracker_filename}. Exiting")
            sys.exit()
    if iteration <= 0 and not release:
        raise AssertionError(f"error parsing metadata file {tracker_filename}")
    if dist.is_initialized():
        t = torch.tensor([iteration], dtype=torch.long,
                         device="cuda" if torch.cuda.is_available() and
                         dist.get_backend() != "gloo" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        max_iter = int(t.item())
        if iteration != max_iter:
            print(f"WARNING: on rank {dist.get_rank()} found iteration {iteration} in the "
                  f"metadata while max iteration across the ranks is {max_iter}, replacing it "
                  "with max iteration.", flush=True)
        iteration = max_iter
    return iteration, release


def get_rng_state():
    args = global_vars.get_args()
    np_state = np.random.get_state()
    rng = {"random_rng_state": random.getstate(),
           "np_rng_state": (np_state[0], torch.from_numpy(np_state[1].copy()),
                            int(np_state[2]), int(np_state[3]), float(np_state[4])),
           "torch_rng_state": torch.get_rng_state(),
           "cuda_rng_state": torch.cuda.get_rng_state() if torch.cuda.is_available() else None,
           "rng_tracker_states": get_cuda_rng_tracker().get_states()}
    states = [rng]
    if dist.is_initialized() and state.get_data_parallel_world_size() > 1 and \
            args.data_parallel_random_init:
        states = [None] * state.get_data_parallel_world_size()
        dist.all_gather_object(states, rng, group=state.get_data_parallel_group())
    return states


def _set_rng_state(rs):
    random.setstate(rs["random_rng_state"])
    nps = rs["np_rng_state"]
    if isinstance(nps, tuple) and torch.is_tensor(nps[1]):
        nps = (nps[0], nps[1].numpy().astype(np.uint32), nps[2], nps[3], nps[4])
    np.random.set_state(nps)
    torch.set_rng_state(rs["torch_rng_state"])
    if torch.cuda.is_available() and rs.get("cuda_rng_state") is not None:
        torch.cuda.set_rng_state(rs["cuda_rng_state"])
    if not rs.get("rng_tracker_states"):
        raise KeyError("rng_tracker_states")
    get_cuda_rng_tracker().set_states(rs["rng_tracker_states"])


def _to_host(obj):
    if torch.is_tensor(obj):
        return obj.detach().to("cpu", non_blocking=False)
    if isinstance(obj, dict):
        return {k: _to_host(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        t = [_to_host(v) for v in obj]
        return type(obj)(t) if not isinstance(obj, tuple) else tuple(t)
    return obj


def wait_for_async_save():
    global _ASYNC_THREAD
    if _ASYNC_THREAD is not None:
        _ASYNC_THREAD.join()
        _ASYNC_THREAD = None


def save_checkpoint(iteration, model, optimizer, opt_param_scheduler):
    args = global_vars.get_args()
    from .parallel import comm  # noqa: PLC0415
    comm.check_xgmi()  # never write weights computed after a timed-out xGMI wait
    if optimizer is not None:
        optimizer.resolve_pending()   # settle a lazily-checked skipped step
        optimizer.wait_param_sync()   # dist-opt parameter all-gather in flight
    model = unwrap_model(model)
    wait_for_async_save()
    print_rank_0(f"saving checkpoint at iteration {iteration:7d} to {args.save}")
    rng_state = get_rng_state() if not args.no_save_rng else None
    model_name, optim_name = get_checkpoint_names(args.save, iteration,
                                                  args.use_distributed_optimizer)
    writes = []
    if args.use_distributed_optimizer and not args.no_save_optim and optimizer is not None:
        writes.append((optim_name, {"optimizer": optimizer.state_dict()}))
    if not dist.is_initialized() or state.get_data_parallel_rank() == 0:
        sd = {"args": args, "checkpoint_version": 3.0, "iteration": iteration}
        if len(model) == 1:
            sd["model"] = model[0].state_dict_for_save_checkpoint()
        else:
            for i, m in enumerate(model):
                state.set_virtual_pipeline_model_parallel_rank(i)
                sd[f"model{i}"] = m.state_dict_for_save_checkpoint()
        if not args.no_save_optim:
            if optimizer is not None and not args.use_distributed_optimizer:
                sd["optimizer"] = optimizer.state_dict()
            if opt_param_scheduler is not None:
                sd["opt_param_scheduler"] = opt_param_scheduler.state_dict()
        if not args.no_save_rng:
            sd["rng_state"] = rng_state
        writes.append((model_name, sd))

    def _write(items):
        for name, obj in items:
            ensure_directory_exists(name)
            # enums pickled under megatron.model.enums: the reference loads these files
            torch.save(obj, name, pickle_module=ckpt_pickle.pickle_module)

    if args.async_save:
        items = [(n, _to_host(o)) for n, o in writes]
        global _ASYNC_THREAD
        _ASYNC_THREAD = threading.Thread(target=_write, args=(items,), daemon=True)
        _ASYNC_THREAD.start()
        wait_for_async_save()  # tracker is written only after data is durable
    else:
        _write(writes)
    if dist.is_initialized():
        dist.barrier()
    print_rank_0(f"  successfully saved checkpoint at iteration {iteration:7d} to {args.save}")
    if not dist.is_initialized() or dist.get_rank() == 0:
        with open(get_checkpoint_tracker_filename(args.save), "w") as f:
            f.write(str(iteration))
    if dist.is_initialized():
        dist.barrier()


def _load_base_checkpoint(load_dir, use_distributed_optimizer, rank0=False):
    tracker = get_checkpoint_tracker_filename(load_dir)
    if not os.path.isfile(tracker):
        if not rank0:
            print_rank_0(f"WARNING: could not find the metadata file {tracker} ")
            print_rank_0("    will not load any checkpoints and will start from random")
        return None, None, False
    iteration, release = read_metadata(tracker) if not rank0 else _read_meta_local(tracker)
    if rank0:
        model_name, optim_name = _rank0_names(load_dir, iteration, use_distributed_optimizer,
                                              release)
    else:
        model_name, optim_name = get_checkpoint_names(load_dir, iteration,
                                                      use_distributed_optimizer, release)
        print_rank_0(f" loading checkpoint from {load_dir} at iteration {iteration}")
    model_sd = safe_load(model_name)
    optim_sd = None
    if use_distributed_optimizer and not rank0:
        if not os.path.exists(optim_name):  # written at a smaller DP size
            optim_name = DPPeerLoader(load_dir, iteration, release).path(0)
        if os.path.exists(optim_name):
            optim_sd = safe_load(optim_name, mmap=True)
    elif not use_distributed_optimizer:
        optim_sd = model_sd
    return model_sd, optim_sd, release


def _read_meta_local(tracker):
    with open(tracker) as f:
        meta = f.read().strip()
    return (0, True) if meta == "release" else (int(meta), False)


def _rank0_names(load_dir, iteration, use_dist_opt, release):
    d = "release" if release else f"iter_{iteration:07d}"
    for sub in ("mp_rank_00", "mp_rank_00_000"):
        name = os.path.join(load_dir, d, sub,
                            "model_rng.pt" if use_dist_opt else "model_optim_rng.pt")
        if os.path.isfile(name):
            return name, name
        alt = os.path.join(load_dir, d, sub, "model_optim_rng.pt")
        if os.path.isfile(alt):
            return alt, alt
    raise FileNotFoundError(f"no rank-0 checkpoint under {os.path.join(load_dir, d)}")


def load_args_from_checkpoint(args, load_arg="load"):
    """--use_checkpoint_args: take model-shape args from the checkpoint."""
    load_dir = getattr(args, load_arg)
    if load_dir is None:
        return args, args
    sd, _, _ = _load_base_checkpoint(load_dir, False, rank0=True)
    if sd is None or "args" not in sd:
        print("Checkpoint not found / has no args to load from", flush=True)
        return args, args
    ck = sd["args"]
    args.iteration = sd["iteration"] if sd.get("iteration") != "release" else 0

    def _set(name, force=False):
        if not force and getattr(args, name, None) is not None:
            return
        v = getattr(ck, name, None)
        if v is not None:
            setattr(args, name, v)

    for n in ("tensor_model_parallel_size", "pipeline_model_parallel_size"):
        _set(n, force=True)
    for n in ("num_layers", "hidden_size", "ffn_hidden_size", "seq_length",
              "num_attention_heads", "num_attention_heads_kv", "kv_channels",
              "max_position_embeddings", "glu_activation", "layernorm_epsilon",
              "rope_scaling_factor"):
        _set(n)
    for n in ("position_embedding_type", "parallel_attn", "parallel_layernorm", "use_rms_norm",
              "tie_embed_logits", "make_vocab_size_divisible_by", "use_bias",
              "padded_vocab_size"):
        _set(n, force=True)
    return args, ck


def _transpose_first_dim(t, num_splits, num_splits_first, heads, head_dim):
    """Row-block reorder of a fused QKV (or KV) weight/bias to the 2.0+ layout
    ``[np, num_splits, hn, ...]`` (reference ``checkpointing.py:340-376``)."""
    shape = t.shape
    if num_splits_first:   # [num_splits * np * hn, ...] (checkpoint_version 0)
        t = t.view(num_splits, heads, head_dim, *shape[1:]).transpose(0, 1)
    else:                  # [np * hn * num_splits, ...] (checkpoint_version 1.0)
        t = t.view(heads, head_dim, num_splits, *shape[1:]).transpose(1, 2)
    return t.contiguous().view(*shape)


def fix_query_key_value_ordering(model, checkpoint_version):
    """Checkpoints older than 2.0 stored fused QKV rows as [3, np, hn] (v0) or
    [np, hn, 3] (v1.0); migrate them in place to the [np, 3, hn] layout
    (reference ``checkpointing.py:379-411``; GQA/MQA weights never had the old
    layouts and are left alone)."""
    if checkpoint_version >= 2.0:
        return
    if checkpoint_version not in (0, 1.0):
        raise ValueError(f"Invalid checkpoint version {checkpoint_version}.")
    if isinstance(model, list):
        if len(model) != 1:
            raise AssertionError("QKV migration supports a single model chunk")
        model = model[0]
    while hasattr(model, "module"):
        model = model.module
    args = global_vars.get_args()
    attn = model.language_model.encoder.layers[0].self_attention
    heads = attn.num_attention_heads_per_partition
    head_dim = attn.hidden_size_per_attention_head
    first = checkpoint_version == 0
    for name, param in model.named_parameters():
        if name.endswith((".query_key_value.weight", ".query_key_value.bias")):
            if args.num_attention_heads_kv != args.num_attention_heads:
                continue
            with torch.no_grad():
                param.copy_(_transpose_first_dim(param.data, 3, first, heads, head_dim))
        elif name.endswith((".key_value.weight", ".key_value.bias")):
            with torch.no_grad():
                param.copy_(_transpose_first_dim(param.data, 2, first, heads, head_dim))
    print_rank_0(f" succesfully fixed query-key-values ordering for checkpoint version "
                 f"{checkpoint_version}")


def load_checkpoint(model, optimizer, opt_param_scheduler, load_arg="load", strict=True):
    args = global_vars.get_args()
    load_dir = getattr(args, load_arg)
    model = unwrap_model(model)
    model_sd, optim_sd, release = _load_base_checkpoint(load_dir, args.use_distributed_optimizer)
    if model_sd is None:
        return 0
    set_checkpoint_version(model_sd.get("checkpoint_version", 0))
    if args.finetune or release:
        iteration = 0
    else:
        iteration = model_sd.get("iteration", model_sd.get("total_iters", 0))
    if "args" in model_sd and not args.finetune:
        ck = model_sd["args"]
        check_checkpoint_args(ck)
        args.consumed_train_samples = getattr(ck, "consumed_train_samples", 0)
        args.consumed_valid_samples = getattr(ck, "consumed_valid_samples", 0)
    if len(model) == 1:
        model[0].load_state_dict(model_sd["model"], strict=strict)
    else:
        for i, m in enumerate(model):
            state.set_virtual_pipeline_model_parallel_rank(i)
            m.load_state_dict(model_sd[f"model{i}"], strict=strict)
    fix_query_key_value_ordering(model[0], get_checkpoint_version())
    decode_pack.bump_weight_generation()  # weights replaced: derived copies are stale
    if optimizer is not None:
        optimizer.reload_model_params()
    if not release and not args.finetune and not args.no_load_optim:
        try:
            if optimizer is not None and (optim_sd is None or "optimizer" not in optim_sd):
                # e.g. a checkpoint written without the distributed optimizer
                # (no optim.pt) or with --no_save_optim: never resume silently
                # with fresh Adam moments
                raise KeyError("optimizer state not found" + (
                    " (no distrib_optim.pt / optim.pt shard for this rank or DP rank 0)"
                    if args.use_distributed_optimizer else ""))
            if optimizer is not None:
                if args.use_distributed_optimizer:
                    it, rel = _read_meta_local(get_checkpoint_tracker_filename(load_dir))
                    optimizer.load_state_dict(optim_sd["optimizer"],
                                              dp_peer_loader=DPPeerLoader(load_dir, it, rel))
                else:
                    optimizer.load_state_dict(optim_sd["optimizer"])
            if opt_param_scheduler is not None and "opt_param_scheduler" in model_sd:
                opt_param_scheduler.load_state_dict(model_sd["opt_param_scheduler"])
        except KeyError as e:
            print_rank_0(f"Unable to load optimizer from checkpoint {load_dir}: {e}. Specify "
                         "--no_load_optim or --finetune to prevent attempting to load the "
                         "optimizer state, exiting ...")
            sys.exit(1)
    if not release and not args.finetune and not args.no_load_rng and "rng_state" in model_sd:
        try:
            rs = model_sd["rng_state"]
            if args.data_parallel_random_init:
                rs = rs[state.get_data_parallel_rank()]
            else:
                rs = rs[0]
            _set_rng_state(rs)
        except KeyError:
            print_rank_0(f"Unable to load rng state from checkpoint {load_dir}. Specify "
                         "--no_load_rng or --finetune to prevent attempting to load the rng "
                         "state, exiting ...")
            sys.exit()
    if dist.is_initialized():
        dist.barrier()
    print_rank_0(f"  successfully loaded checkpoint from {load_dir} at iteration {iteration}")
    return iteration


def load_biencoder_checkpoint(model, only_query_model=False, only_context_model=False,
                              custom_load_path=None):
    """Load just the retriever tower(s) needed for indexing / retrieval
    (reference megatron/checkpointing.py:689-730; the reference reads an
    undefined ``model_checkpoint_name`` there, here the resolved name is used
    and ``release`` trackers are accepted)."""
    from .utils.misc import unwrap_model
    args = global_vars.get_args()
    model = unwrap_model(model)
    load_path = custom_load_path if custom_load_path is not None else args.load
    iteration, release = _read_meta_local(get_checkpoint_tracker_filename(load_path))
    name, _ = get_checkpoint_names(load_path, iteration, args.use_distributed_optimizer,
                                   release=release)
    if state.get_data_parallel_rank() == 0:
        print(f"global rank {dist.get_rank() if dist.is_initialized() else 0} is loading "
              f"checkpoint {name}", flush=True)
    sd = dict(safe_load(name)["model"])
    if only_query_model:
        sd.pop("context_model", None)
    if only_context_model:
        sd.pop("query_model", None)
    assert len(model) == 1
    model[0].load_state_dict(sd)
    if dist.is_initialized():
        dist.barrier()
    if state.get_data_parallel_rank() == 0:
        print(f" successfully loaded {name}", flush=True)
    return model

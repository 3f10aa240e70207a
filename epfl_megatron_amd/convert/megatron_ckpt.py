"""Read / write whole Megatron checkpoints on disk without a process group.

``load_full(dir)`` memory-maps every ``mp_rank_TT[_PPP]/model_optim_rng.pt``
(``torch.load(mmap=True, weights_only=True)``: tensors stay on disk until
touched, so re-sharding a 70B model does not need 2x its size in RAM) and
merges the TP x PP shards into the canonical full dict of :mod:`.shard`.
``save_sharded`` writes any TP x PP layout of the same dict, with a tracker
file, in the layout of SURVEY Appendix B.
"""
import argparse
import os

import torch

from .. import ckpt_pickle
from ..checkpointing import _safe_globals
from .shard import merge_shards, split_full

TRACKER = "latest_checkpointed_iteration.txt"


def read_tracker(ckpt_dir):
    with open(os.path.join(ckpt_dir, TRACKER)) as f:
        return f.read().strip()


def iteration_dir(ckpt_dir, iteration):
    it = str(iteration)
    return os.path.join(ckpt_dir, "release" if it == "release" else f"iter_{int(it):07d}")


def shard_name(tp_rank, pp_rank, pp_size):
    return f"mp_rank_{tp_rank:02d}" if pp_size == 1 else f"mp_rank_{tp_rank:02d}_{pp_rank:03d}"


def _load(path):
    with torch.serialization.safe_globals(_safe_globals()):
        try:
            return torch.load(path, map_location="cpu", weights_only=True, mmap=True)
        except RuntimeError:  # legacy (non-zip) serialization cannot be mapped
            return torch.load(path, map_location="cpu", weights_only=True)


def _shard_file(d):
    for name in ("model_optim_rng.pt", "model_rng.pt"):
        if os.path.isfile(os.path.join(d, name)):
            return os.path.join(d, name)
    raise FileNotFoundError(f"no model file in {d}")


def load_full(ckpt_dir, iteration=None):
    """-> (args Namespace, full canonical dict, iteration string)."""
    iteration = iteration or read_tracker(ckpt_dir)
    base = iteration_dir(ckpt_dir, iteration)
    first = _load(_shard_file(os.path.join(base, "mp_rank_00"))) \
        if os.path.isdir(os.path.join(base, "mp_rank_00")) else \
        _load(_shard_file(os.path.join(base, "mp_rank_00_000")))
    args = first["args"]
    tp = getattr(args, "tensor_model_parallel_size", 1) or 1
    pp = getattr(args, "pipeline_model_parallel_size", 1) or 1
    if pp > 1 and not os.path.isdir(os.path.join(base, shard_name(0, 0, pp))):
        pp = 1
    shards = [[None] * tp for _ in range(pp)]
    for p in range(pp):
        for r in range(tp):
            sd = first if (p == 0 and r == 0) else \
                _load(_shard_file(os.path.join(base, shard_name(r, p, pp))))
            if "model" not in sd:
                raise ValueError("virtual-pipeline checkpoints (model0, model1, ...) must be "
                                 "re-saved without interleaving before conversion")
            shards[p][r] = sd["model"]
    num_layers = getattr(args, "num_layers", None) or getattr(args, "encoder_num_layers")
    glu = bool(getattr(args, "glu_activation", None))
    return args, merge_shards(shards, num_layers, glu), iteration


def _own(obj):
    """Deep copy with every tensor compacted (chunks are views of the full
    tensor; saving a view would write the whole storage)."""
    if isinstance(obj, dict):
        return {k: _own(v) for k, v in obj.items()}
    if torch.is_tensor(obj):
        return obj.contiguous().clone()
    return obj


def save_sharded(ckpt_dir, full, args, tp=1, pp=1, iteration="release", padded_vocab=None,
                 checkpoint_version=3.0):
    """Write ``full`` as a TP x PP checkpoint; ``args`` is stored in every shard."""
    args = argparse.Namespace(**vars(args))
    args.tensor_model_parallel_size = tp
    args.pipeline_model_parallel_size = pp
    if padded_vocab is not None:
        args.padded_vocab_size = padded_vocab
    shards = split_full(full, tp, pp, args.num_layers, bool(getattr(args, "glu_activation", None)),
                        bool(getattr(args, "tie_embed_logits", True)), padded_vocab)
    base = iteration_dir(ckpt_dir, iteration)
    for p in range(pp):
        for r in range(tp):
            d = os.path.join(base, shard_name(r, p, pp))
            os.makedirs(d, exist_ok=True)
            model = _own(shards[p][r])
            torch.save({"iteration": iteration if iteration == "release" else int(iteration),
                        "model": model, "checkpoint_version": checkpoint_version,
                        "args": args}, os.path.join(d, "model_optim_rng.pt"),
                       pickle_module=ckpt_pickle.pickle_module)
    with open(os.path.join(ckpt_dir, TRACKER), "w") as f:
        f.write(str(iteration))
    return base

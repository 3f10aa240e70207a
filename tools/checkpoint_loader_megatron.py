"""Loader plugin: any-TP x PP Megatron checkpoint -> (metadata, full canonical dict).

Reference: ``tools/checkpoint_loader_megatron.py`` (fakes a TP/PP topology and
instantiates the model per shard); here shards are merged as state dicts by
the rules of ``epfl_megatron_amd.convert.shard`` without building a model.
"""
import argparse

import torch


def add_arguments(parser):
    g = parser.add_argument_group(title="Megatron loader")
    g.add_argument("--true_vocab_size", type=int, default=None,
                   help="original vocab size; padding is recomputed for the target TP")
    g.add_argument("--vocab_file", type=str, default=None,
                   help="tokenizer model to derive the true vocab size from")
    g.add_argument("--megatron_path", type=str, default=None, help="(ignored)")


def _true_vocab(args, margs):
    if args.true_vocab_size is not None:
        return args.true_vocab_size
    if args.vocab_file is not None:
        from epfl_megatron_amd.tokenizer import build_tokenizer
        a = argparse.Namespace(**vars(margs))
        a.vocab_file = args.vocab_file
        a.rank = 0
        a.tensor_model_parallel_size = 1
        a.make_vocab_size_divisible_by = 1
        for k, v in (("vocab_extra_ids", 0), ("vocab_extra_ids_list", None),
                     ("new_tokens", True), ("tokenizer_model", None), ("merge_file", None),
                     ("synthetic_vocab_size", 0)):
            if not hasattr(a, k):
                setattr(a, k, v)
        return build_tokenizer(a).vocab_size
    return None


def load_checkpoint(args):
    from epfl_megatron_amd.convert.megatron_ckpt import load_full
    margs, full, iteration = load_full(args.load_dir)
    if getattr(args, "bf16", False):
        full = {k: ({kk: vv.to(torch.bfloat16) for kk, vv in v.items()} if isinstance(v, dict)
                    else v.to(torch.bfloat16)) for k, v in full.items()}
    md = argparse.Namespace(margs=margs, iteration=iteration, true_vocab_size=_true_vocab(args, margs),
                            tie_embed_logits="lm_head" not in full,
                            model_type=args.model_type)
    print(f"loaded {args.load_dir}: TP={margs.tensor_model_parallel_size} "
          f"PP={margs.pipeline_model_parallel_size}, {margs.num_layers} layers")
    return md, full

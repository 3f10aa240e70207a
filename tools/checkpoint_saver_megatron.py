"""Saver plugin: full canonical dict -> Megatron checkpoint at the target TP x PP.

Reference: ``tools/checkpoint_saver_megatron.py``.  The vocab is re-padded
for the target TP (``make_vocab_size_divisible_by x TP``) when the true vocab
size is known, trimming or replicating the last row as the reference does.
"""


def add_arguments(parser):
    g = parser.add_argument_group(title="Megatron saver")
    g.add_argument("--megatron_path", type=str, default=None, help="(ignored)")
    g.add_argument("--target_tensor_parallel_size", type=int, default=None,
                   help="target TP size (default: the source's)")
    g.add_argument("--target_pipeline_parallel_size", type=int, default=None,
                   help="target PP size (default: the source's)")


def save_checkpoint(args, md, full):
    from epfl_megatron_amd.convert.megatron_ckpt import save_sharded
    margs = md.margs
    tp = args.target_tensor_parallel_size or margs.tensor_model_parallel_size
    pp = args.target_pipeline_parallel_size or margs.pipeline_model_parallel_size
    nkv = getattr(margs, "num_attention_heads_kv", None) or margs.num_attention_heads
    if nkv % tp:
        raise ValueError(f"num_attention_heads_kv={nkv} is not divisible by TP={tp}")
    padded = None
    if md.true_vocab_size is not None:
        mult = (getattr(margs, "make_vocab_size_divisible_by", 128) or 1) * tp
        padded = -(-md.true_vocab_size // mult) * mult
    else:
        rows = full["embedding"]["word_embeddings.weight"].shape[0]
        if rows % tp:
            raise ValueError(f"vocab rows {rows} not divisible by TP={tp}; pass "
                             "--true_vocab_size or --vocab_file")
        print("Original vocab size not specified, leaving embedding table as-is.")
    out = save_sharded(args.save_dir, full, margs, tp=tp, pp=pp, iteration=md.iteration,
                       padded_vocab=padded)
    print(f"saved TP={tp} PP={pp} checkpoint to {out}")

"""Megatron checkpoint -> Hugging Face Llama / Falcon model directory.

Reference CLI (``weights2megatron/megatron2hf.py:434-471``)::

    python weights2megatron/megatron2hf.py --model {llama,llama2,falcon} \
        --input_dir CKPT --output_dir HF_DIR [--vocab_file tokenizer.model] \
        [--num_output_shards N] [--vocab_extra_ids_list ...] [--override_special_tokens k=v ...]

Unlike the reference, any TP x PP sharding is accepted (shards are merged in
memory-mapped form; the reference required TP = PP = 1).  The padded vocab is
kept (as the reference does) so that Megatron special tokens map to the same
ids.  The tokenizer is written from ``--vocab_file`` (a SentencePiece model,
or ``tokenizer.model`` next to the checkpoint); Falcon tokenizers need a local
``--vocab_file`` directory (no network access here).
"""
import argparse
import os
import sys
import warnings

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), os.path.pardir)))

from epfl_megatron_amd.convert.falcon import megatron_to_hf_falcon  # noqa: E402
from epfl_megatron_amd.convert.llama import megatron_to_hf_llama  # noqa: E402
from epfl_megatron_amd.convert.megatron_ckpt import load_full  # noqa: E402


def _dtype_of(sd):
    return next(iter(sd.values())).dtype


def write_llama_model(model_path, input_base_path, num_output_shards=1, norm_eps=None):
    from transformers import LlamaConfig, LlamaForCausalLM
    args, full, _ = load_full(input_base_path)
    heads = args.num_attention_heads
    kv = getattr(args, "num_attention_heads_kv", None) or heads
    sd = megatron_to_hf_llama(full, heads, kv)
    cfg = LlamaConfig(vocab_size=sd["model.embed_tokens.weight"].shape[0],
                      hidden_size=args.hidden_size, intermediate_size=args.ffn_hidden_size,
                      num_attention_heads=heads, num_key_value_heads=kv,
                      num_hidden_layers=args.num_layers,
                      rms_norm_eps=norm_eps or getattr(args, "layernorm_epsilon", 1e-5),
                      max_position_embeddings=args.seq_length,
                      tie_word_embeddings=False)
    _save_hf(LlamaForCausalLM, cfg, sd, model_path, num_output_shards)


def write_falcon_model(model_path, input_base_path, num_output_shards=1):
    from transformers import FalconConfig, FalconForCausalLM
    args, full, _ = load_full(input_base_path)
    heads = args.num_attention_heads
    kv = getattr(args, "num_attention_heads_kv", None) or heads
    sd = megatron_to_hf_falcon(full, heads, kv)
    new_arch = any(".ln_attn." in k for k in sd)
    cfg = FalconConfig(vocab_size=sd["transformer.word_embeddings.weight"].shape[0],
                       hidden_size=args.hidden_size, num_hidden_layers=args.num_layers,
                       num_attention_heads=heads, num_kv_heads=kv if new_arch else None,
                       new_decoder_architecture=new_arch, multi_query=(kv == 1),
                       parallel_attn=True, bias=False,
                       layer_norm_epsilon=getattr(args, "layernorm_epsilon", 1e-5))
    _save_hf(FalconForCausalLM, cfg, sd, model_path, num_output_shards)


def _save_hf(cls, cfg, sd, model_path, num_output_shards):
    dtype = _dtype_of(sd)
    with torch.device("meta"):
        model = cls(cfg)
    model.load_state_dict(sd, strict=False, assign=True)
    missing = [n for n, p in model.named_parameters() if p.is_meta]
    if missing:
        raise KeyError(f"conversion left parameters unset: {missing[:5]}")
    model.to(dtype)
    nbytes = sum(v.numel() * v.element_size() for v in sd.values())
    shard = max(nbytes // max(num_output_shards, 1) + 1, 1 << 20)
    model.save_pretrained(model_path, max_shard_size=shard, safe_serialization=True)
    print(f"Saved {cls.__name__} ({dtype}) to {model_path}")


def write_tokenizer(args):
    """SentencePiece tokenizer with the Megatron special tokens appended at the
    same ids (reference megatron2hf.py:352-431)."""
    from epfl_megatron_amd.tokenizer import build_tokenizer
    if args.model in {"llama", "llama2"}:
        from transformers import LlamaTokenizer
        vocab = args.vocab_file or os.path.join(args.input_dir, "tokenizer.model")
        if not os.path.isfile(vocab):
            warnings.warn("no tokenizer.model found; skipping the tokenizer")
            return None
        hf_tok = LlamaTokenizer(vocab_file=vocab, legacy=True)
        args.vocab_file = vocab
        args.tokenizer_type = "SentencePieceTokenizer"
    else:
        if not args.vocab_file:
            warnings.warn("Falcon tokenizer needs a local --vocab_file directory; skipping")
            return None
        from transformers import AutoTokenizer
        hf_tok = AutoTokenizer.from_pretrained(args.vocab_file)
        args.tokenizer_type = "FalconTokenizer"
    args.rank, args.vocab_extra_ids, args.new_tokens = 0, 0, True
    args.make_vocab_size_divisible_by, args.tensor_model_parallel_size = 128, 1
    args.tokenizer_model = None
    mt = build_tokenizer(args)
    if args.tokenizer_type == "SentencePieceTokenizer":
        for name, tok in (("cls", "<CLS>"), ("sep", "<SEP>"), ("eod", "<EOD>"),
                          ("mask", "<MASK>"), ("pad", "<PAD>")):
            if getattr(mt, name, None) is not None:
                hf_tok.add_tokens(tok, special_tokens=True)
                if name != "eod":
                    setattr(hf_tok, f"{name}_token", tok)
        extra = list(args.vocab_extra_ids_list.split(",")) if args.vocab_extra_ids_list else []
        if extra:
            hf_tok.add_special_tokens({"additional_special_tokens": extra})
        hf_vocab = hf_tok.get_vocab()
        for t in ["<CLS>", "<SEP>", "<EOD>", "<MASK>", "<PAD>"] + extra:
            if t in mt.vocab and mt.vocab.get(t) != hf_vocab.get(t):
                raise AssertionError(f"megatron/HF tokenizer id mismatch for {t}: "
                                     f"{mt.vocab.get(t)} vs {hf_vocab.get(t)}")
    for override in args.override_special_tokens or []:
        try:
            key, value = override.split("=")
            if key not in {"bos", "cls", "eos", "mask", "pad", "sep", "unk"}:
                raise AssertionError
            if value not in mt.vocab:
                raise KeyError(value)
            setattr(hf_tok, f"{key}_token", value)
        except ValueError:
            warnings.warn(f"Illegal override string {override}")
        except AssertionError:
            warnings.warn(f"Cannot override key {override}")
        except KeyError:
            warnings.warn(f"Token {override} not found in megatron tokenizer")
    hf_tok.save_pretrained(args.output_dir)
    return hf_tok


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--input_dir", required=True, help="Megatron checkpoint directory")
    p.add_argument("--num_output_shards", type=int, default=1)
    p.add_argument("--model", choices={"falcon", "llama", "llama2"}, default="llama2")
    p.add_argument("--output_dir", required=True)
    p.add_argument("--cache_dir", help="(unused: no network access)")
    p.add_argument("--vocab_file", type=str)
    p.add_argument("--vocab_extra_ids_list")
    p.add_argument("--override_special_tokens", nargs="*", default=[])
    p.add_argument("--no_tokenizer", action="store_true")
    args = p.parse_args(argv)
    if args.model in {"llama", "llama2"}:
        write_llama_model(args.output_dir, args.input_dir, args.num_output_shards)
    else:
        write_falcon_model(args.output_dir, args.input_dir, args.num_output_shards)
    if not args.no_tokenizer:
        write_tokenizer(args)


if __name__ == "__main__":
    main()

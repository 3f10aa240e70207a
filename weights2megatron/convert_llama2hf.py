"""Meta Llama (``consolidated.NN.pth`` + ``params.json``) -> Hugging Face directory
(reference ``weights2megatron/convert_llama2hf.py``; used to produce the HF
baseline for ``verify_correctness.py``).

    python weights2megatron/convert_llama2hf.py --input_dir LLAMA_ROOT --model_size 7B \
        --output_dir HF_DIR [--num_output_shards 2]

Shards are merged with the Meta model-parallel rules, routed through this
framework's canonical dict (``convert.llama``) and written as
``LlamaForCausalLM`` weights; Q/K rows go from Meta's interleaved RoPE pairs
to HF's rotate-half layout.  Shapes come from the tensors (FFN width, KV
heads), ``params.json`` supplies eps / rope_theta.  ``tokenizer.model`` in
``--input_dir`` is copied into the output as a ``LlamaTokenizer``.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), os.path.pardir)))

from epfl_megatron_amd.convert.hf_io import load_meta_shards, meta_params  # noqa: E402
from epfl_megatron_amd.convert.llama import (llama_to_megatron, megatron_to_hf_llama,  # noqa: E402
                                             merge_meta_shards, num_layers_of)

_SIZES = ["7B", "7Bf", "13B", "13Bf", "30B", "34B", "65B", "70B", "70Bf", "tokenizer_only"]


def compute_intermediate_size(n, ffn_dim_multiplier=1, multiple_of=256):
    """Meta's FFN width rule (only used to cross-check the tensors)."""
    return multiple_of * ((int(ffn_dim_multiplier * int(8 * n / 3)) + multiple_of - 1)
                          // multiple_of)


def write_model(model_path, input_base_path, num_output_shards=2, safe_serialization=True):
    from transformers import LlamaConfig, LlamaForCausalLM
    params = meta_params(input_base_path)
    meta = merge_meta_shards(load_meta_shards(input_base_path))
    vocab, dim = meta["tok_embeddings.weight"].shape
    n_heads = params.get("n_heads")
    head_dim = dim // n_heads
    n_kv = meta["layers.0.attention.wk.weight"].shape[0] // head_dim
    ffn = meta["layers.0.feed_forward.w1.weight"].shape[0]
    if "multiple_of" in params:
        want = compute_intermediate_size(dim, params.get("ffn_dim_multiplier") or 1,
                                         params["multiple_of"])
        if want != ffn:
            print(f"note: params.json implies ffn {want}, tensors have {ffn}; using tensors")
    full = llama_to_megatron(meta, n_heads, n_kv, source="meta")
    sd = megatron_to_hf_llama(full, n_heads, n_kv)
    cfg = LlamaConfig(vocab_size=vocab, hidden_size=dim, intermediate_size=ffn,
                      num_attention_heads=n_heads, num_key_value_heads=n_kv,
                      num_hidden_layers=num_layers_of(meta),
                      rms_norm_eps=params.get("norm_eps", 1e-5),
                      rope_theta=params.get("rope_theta", 10000.0),
                      max_position_embeddings=params.get("max_seq_len", 4096 if n_kv != n_heads
                                                         or dim >= 4096 else 2048),
                      tie_word_embeddings=False)
    dtype = meta["tok_embeddings.weight"].dtype
    with torch.device("meta"):
        model = LlamaForCausalLM(cfg)
    model.load_state_dict(sd, strict=False, assign=True)
    unset = [n for n, p in model.named_parameters() if p.is_meta]
    if unset:
        raise KeyError(f"conversion left parameters unset: {unset[:5]}")
    model.to(dtype)
    nbytes = sum(v.numel() * v.element_size() for v in sd.values())
    model.save_pretrained(model_path, safe_serialization=safe_serialization,
                          max_shard_size=max(nbytes // max(num_output_shards, 1) + 1, 1 << 20))
    print(f"Saved LlamaForCausalLM ({dtype}, {cfg.num_hidden_layers} layers) to {model_path}")


def write_tokenizer(tokenizer_path, input_tokenizer_path):
    if not os.path.isfile(input_tokenizer_path):
        print(f"no tokenizer at {input_tokenizer_path}; skipping")
        return
    from transformers import LlamaTokenizer
    LlamaTokenizer(vocab_file=input_tokenizer_path).save_pretrained(tokenizer_path)
    print(f"Saved tokenizer to {tokenizer_path}")


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--input_dir", required=True,
                   help="LLaMA root (tokenizer.model + per-size folders) or a shard folder")
    p.add_argument("--model_size", choices=_SIZES, default=None)
    p.add_argument("--num_output_shards", type=int, default=2)
    p.add_argument("--output_dir", required=True)
    p.add_argument("--safe_serialization", type=lambda s: s.lower() not in ("0", "false", "no"),
                   default=True)
    args = p.parse_args(argv)
    if args.model_size != "tokenizer_only":
        src = args.input_dir if args.model_size is None else \
            os.path.join(args.input_dir, args.model_size)
        write_model(args.output_dir, src, args.num_output_shards, args.safe_serialization)
    write_tokenizer(args.output_dir, os.path.join(args.input_dir, "tokenizer.model"))


if __name__ == "__main__":
    main()

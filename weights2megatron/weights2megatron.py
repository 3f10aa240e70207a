"""Meta / Hugging Face weights -> a Megatron ``release`` checkpoint.

Reference CLI (``weights2megatron/weights2megatron.py:226-261``)::

    python weights2megatron/weights2megatron.py {falcon,llama,llama2,codellama} \
        --size 7 --out OUT_DIR --cache-dir WEIGHTS_DIR

``--cache-dir`` (alias ``--model-path``) is a local directory: a Meta
checkpoint (``consolidated.NN.pth`` + ``params.json``) or a Hugging Face
snapshot (``config.json`` + safetensors/bin).  There is no network access, so
nothing is downloaded.  Output: ``OUT/latest_checkpointed_iteration.txt`` =
``release`` and ``OUT/release/mp_rank_00/model_optim_rng.pt`` with
``checkpoint_version`` 3.0 and the training args; for HF
Llama sources the ``tokenizer.model`` is copied next to it.  Re-shard with
``tools/checkpoint_util.py``.
"""
import argparse
import os
import shutil
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), os.path.pardir)))

from epfl_megatron_amd.convert import hf_io  # noqa: E402
from epfl_megatron_amd.convert.falcon import falcon_args, falcon_to_megatron  # noqa: E402
from epfl_megatron_amd.convert.llama import (SIZES, hf_to_meta, llama_args,  # noqa: E402
                                             llama_to_megatron, merge_meta_shards)
from epfl_megatron_amd.convert.megatron_ckpt import save_sharded  # noqa: E402


def convert_llama(src, size, version):
    if hf_io.is_meta_dir(src):
        weights = merge_meta_shards(hf_io.load_meta_shards(src))
        params = hf_io.meta_params(src)
        source = "meta"
        heads = params.get("n_heads")
        kv = params.get("n_kv_heads")
        eps = params.get("norm_eps")
    else:
        weights = hf_to_meta(hf_io.load_hf_state_dict(src))
        cfg = hf_io.hf_config(src)
        source = "hf"
        heads = cfg.get("num_attention_heads")
        kv = cfg.get("num_key_value_heads")
        eps = cfg.get("rms_norm_eps")
    known = SIZES.get(size)
    layers = max(int(k.split(".")[1]) for k in weights if k.startswith("layers.")) + 1
    hidden = weights["tok_embeddings.weight"].shape[1]
    vocab = weights["tok_embeddings.weight"].shape[0]
    ffn = weights["layers.0.feed_forward.w1.weight"].shape[0]
    heads = heads or (known[2] if known else None)
    if heads is None:
        raise ValueError("number of attention heads unknown: provide params.json/config.json")
    if kv is None:
        kv = known[4] if (known and version == 2) else heads
    full = llama_to_megatron(weights, heads, kv, source)
    args = llama_args(layers, hidden, heads, ffn, kv, version=version, vocab=vocab, norm_eps=eps)
    if version == 3:  # Code Llama: 16k context, rope theta 1e6
        args.update(max_position_embeddings=16384, seq_length=16384, rope_theta=1e6)
    return full, args, source


def convert_falcon(src):
    sd = hf_io.load_hf_state_dict(src)
    cfg = hf_io.hf_config(src)
    heads = cfg.get("num_attention_heads") or cfg.get("n_head")
    new_arch = cfg.get("new_decoder_architecture", any(".ln_attn." in k for k in sd))
    kv = (cfg.get("num_kv_heads") or cfg.get("n_head_kv") or 1) if new_arch else \
        (1 if cfg.get("multi_query", True) else heads)
    full = falcon_to_megatron(sd, heads, kv)
    layers = cfg.get("num_hidden_layers") or cfg.get("n_layer")
    emb = full["embedding"]["word_embeddings.weight"]
    args = falcon_args(layers, emb.shape[1], heads, kv, vocab=emb.shape[0],
                       parallel_layernorm=any(".ln_attn." in k for k in sd))
    args["layernorm_epsilon"] = cfg.get("layer_norm_epsilon", 1e-5)
    return full, args


def main(model_name="falcon", size=7, out=None, cache_dir=None):
    import argparse as ap
    if cache_dir is None:
        raise ValueError("--cache-dir/--model-path: local directory with the source weights")
    out = out or os.path.abspath(f"{model_name}{size}b_megatron")
    if model_name == "falcon":
        full, args = convert_falcon(str(cache_dir))
        source = "hf"
    else:
        version = {"llama": 1, "llama2": 2, "codellama": 3}[model_name]
        full, args, source = convert_llama(str(cache_dir), size, version)
    args.update(tensor_model_parallel_size=1, pipeline_model_parallel_size=1,
                iteration="release", bias_gelu_fusion=False, bias_dropout_fusion=False,
                position_embedding_type="rotary", model_name=model_name)
    from epfl_megatron_amd.models.enums import PositionEmbeddingType
    args["position_embedding_type"] = PositionEmbeddingType.rotary
    save_sharded(str(out), full, ap.Namespace(**args), tp=1, pp=1, iteration="release")
    print("Saved weights in", out)
    tok = os.path.join(str(cache_dir), "tokenizer.model")
    if model_name != "falcon" and os.path.isfile(tok):
        shutil.copy(tok, os.path.join(str(out), "tokenizer.model"))
        print("Saved tokenizer.model in", os.path.join(str(out), "tokenizer.model"))
    print("Done")
    return out


if __name__ == "__main__":
    p = argparse.ArgumentParser(description="Convert Meta/HF Llama or Falcon weights to a "
                                            "Megatron checkpoint")
    p.add_argument("model", choices={"falcon", "llama", "llama2", "codellama"})
    p.add_argument("--size", default=7, type=int, choices={7, 13, 30, 34, 40, 65, 70})
    p.add_argument("--out", type=str, help="output checkpoint directory")
    p.add_argument("--cache-dir", "--model-path", dest="cache_dir", type=str,
                   help="local directory with the Meta or HF weights")
    p.add_argument("--megatron-path", type=str, help="(ignored; kept for CLI compatibility)")
    a = p.parse_args()
    main(a.model, a.size, a.out, a.cache_dir)

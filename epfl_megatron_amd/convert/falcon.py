"""Falcon (7B multi-query / 40B new decoder architecture) <-> Megatron.

Reference: ``weights2megatron/weights2megatron.py:23-77`` and
``weights2megatron/megatron2hf.py:209-347``.  HF's fused QKV already uses the
grouped ``[q.., k, v]`` per-KV-head layout (multi-query = one group), so only
the rotate-half -> interleaved RoPE permutation is applied.  The two
architectures differ in their norms: 7B has one ``input_layernorm`` shared by
the parallel attention and MLP; 40B has ``ln_attn``/``ln_mlp`` which map to
``input_layernorm``/``mlp_layernorm`` (``--parallel_layernorm``).  The
architecture is detected from the keys, not from the model size.
"""
import torch

from .llama import num_layers_of
from .qkv import permute_qkv


def falcon_to_megatron(hf_sd, n_heads, n_heads_kv):
    emb = hf_sd["transformer.word_embeddings.weight"]
    dim = emb.shape[1]
    if "lm_head.weight" in hf_sd and not torch.equal(hf_sd["lm_head.weight"], emb):
        raise ValueError("Falcon checkpoints tie lm_head to the word embeddings")
    tr = {"final_layernorm.weight": hf_sd["transformer.ln_f.weight"],
          "final_layernorm.bias": hf_sd["transformer.ln_f.bias"]}
    for i in range(num_layers_of(hf_sd, r"^transformer\.h\.(\d+)\.")):
        p, h = f"layers.{i}", f"transformer.h.{i}"
        tr[f"{p}.attention.query_key_value.weight"] = permute_qkv(
            hf_sd[f"{h}.self_attention.query_key_value.weight"], dim, n_heads, n_heads_kv)
        tr[f"{p}.attention.dense.weight"] = hf_sd[f"{h}.self_attention.dense.weight"]
        tr[f"{p}.mlp.dense_h_to_4h.weight"] = hf_sd[f"{h}.mlp.dense_h_to_4h.weight"]
        tr[f"{p}.mlp.dense_4h_to_h.weight"] = hf_sd[f"{h}.mlp.dense_4h_to_h.weight"]
        if f"{h}.ln_attn.weight" in hf_sd:
            for ours, theirs in (("input_layernorm", "ln_attn"), ("mlp_layernorm", "ln_mlp")):
                tr[f"{p}.{ours}.weight"] = hf_sd[f"{h}.{theirs}.weight"]
                tr[f"{p}.{ours}.bias"] = hf_sd[f"{h}.{theirs}.bias"]
        else:
            tr[f"{p}.input_layernorm.weight"] = hf_sd[f"{h}.input_layernorm.weight"]
            tr[f"{p}.input_layernorm.bias"] = hf_sd[f"{h}.input_layernorm.bias"]
    return {"embedding": {"word_embeddings.weight": emb}, "transformer": tr}


def megatron_to_hf_falcon(full, n_heads, n_heads_kv, vocab_size=None):
    tr = full["transformer"]
    emb = full["embedding"]["word_embeddings.weight"]
    v = vocab_size or emb.shape[0]
    dim = emb.shape[1]
    out = {"transformer.word_embeddings.weight": emb[:v], "lm_head.weight": emb[:v],
           "transformer.ln_f.weight": tr["final_layernorm.weight"],
           "transformer.ln_f.bias": tr["final_layernorm.bias"]}
    for i in range(num_layers_of(tr)):
        p, h = f"layers.{i}", f"transformer.h.{i}"
        out[f"{h}.self_attention.query_key_value.weight"] = permute_qkv(
            tr[f"{p}.attention.query_key_value.weight"], dim, n_heads, n_heads_kv, revert=True)
        out[f"{h}.self_attention.dense.weight"] = tr[f"{p}.attention.dense.weight"]
        out[f"{h}.mlp.dense_h_to_4h.weight"] = tr[f"{p}.mlp.dense_h_to_4h.weight"]
        out[f"{h}.mlp.dense_4h_to_h.weight"] = tr[f"{p}.mlp.dense_4h_to_h.weight"]
        if f"{p}.mlp_layernorm.weight" in tr:
            for ours, theirs in (("input_layernorm", "ln_attn"), ("mlp_layernorm", "ln_mlp")):
                out[f"{h}.{theirs}.weight"] = tr[f"{p}.{ours}.weight"]
                out[f"{h}.{theirs}.bias"] = tr[f"{p}.{ours}.bias"]
        else:
            out[f"{h}.input_layernorm.weight"] = tr[f"{p}.input_layernorm.weight"]
            out[f"{h}.input_layernorm.bias"] = tr[f"{p}.input_layernorm.bias"]
    return out


def falcon_args(num_layers, hidden, heads, kv_heads, vocab=65024, parallel_layernorm=None,
                seq_length=2048):
    """Training args of a converted Falcon (reference weights2megatron.py:175-185)."""
    return dict(num_layers=num_layers, hidden_size=hidden, num_attention_heads=heads,
                num_attention_heads_kv=kv_heads, parallel_attn=True,
                parallel_layernorm=bool(parallel_layernorm if parallel_layernorm is not None
                                        else kv_heads > 1),
                tokenizer_type="FalconTokenizer", use_flash_attn=True, hidden_dropout=0.0,
                max_position_embeddings=seq_length, seq_length=seq_length,
                padded_vocab_size=vocab, make_vocab_size_divisible_by=1,
                tie_embed_logits=True, use_bias=False, glu_activation=None,
                use_rms_norm=False, ffn_hidden_size=4 * hidden)

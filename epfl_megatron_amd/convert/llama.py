"""Llama-1/2 (and Code Llama) weights <-> Megatron canonical dict.

Reference behaviour: ``weights2megatron/weights2megatron.py:80-145`` (Meta/HF
-> Megatron), ``weights2megatron/merge_llama.py`` (Meta shard merge, HF key
renames), ``weights2megatron/megatron2hf.py:60-199`` (Megatron -> HF).

* QKV: grouped per KV head (:mod:`.qkv`); HF rows are rotate-half so they are
  permuted to the interleaved RoPE convention on the way in, and back out.
* MLP: ``dense_h_to_4h = cat([w3 (up), w1 (gate)])`` — first half "up",
  second half the SiLU-gated one (GLU convention).
* Shapes (layers, heads, hidden) are inferred from the tensors; the size
  tables below only fill in the training args of known checkpoints.
"""
import re

import torch

from .qkv import pack_qkv, permute_qkv, unpack_qkv

# Published configurations (reference weights2megatron.py:16-20; 34B = Code Llama).
SIZES = {  # size: (layers, hidden, heads, ffn, kv_heads(llama2))
    7: (32, 4096, 32, 11008, 32),
    13: (40, 5120, 40, 13824, 40),
    30: (60, 6656, 52, 17920, 52),
    34: (48, 8192, 64, 22016, 8),
    65: (80, 8192, 64, 22016, 64),
    70: (80, 8192, 64, 28672, 8),
}

# Meta shard concatenation axis per parameter kind (reference merge_llama.py:21-35).
META_SHARD_DIM = {"w1": 0, "w2": -1, "w3": 0, "wo": -1, "wq": 0, "wk": 0, "wv": 0,
                  "output": 0, "tok_embeddings": -1, "ffn_norm": None,
                  "attention_norm": None, "norm": None, "rope": None}

_HF_TO_META = {"self_attn.q_proj": "attention.wq", "self_attn.k_proj": "attention.wk",
               "self_attn.v_proj": "attention.wv", "self_attn.o_proj": "attention.wo",
               "mlp.gate_proj": "feed_forward.w1", "mlp.down_proj": "feed_forward.w2",
               "mlp.up_proj": "feed_forward.w3", "input_layernorm": "attention_norm",
               "post_attention_layernorm": "ffn_norm"}
_META_TO_HF = {v: k for k, v in _HF_TO_META.items()}


def merge_meta_shards(shards):
    """Meta ``consolidated.NN.pth`` state dicts (model-parallel shards) -> one dict."""
    if len(shards) == 1:
        return dict(shards[0])
    out = {}
    for name in shards[0]:
        kind = name.split(".")[-2]
        dim = META_SHARD_DIM[kind]
        if dim is None:
            out[name] = shards[0][name]
        else:
            out[name] = torch.cat([s[name] for s in shards], dim=dim)
    return out


def hf_to_meta(sd):
    """Rename HF Llama keys to Meta keys (reference merge_llama.py:89-109)."""
    out = {}
    for k, v in sd.items():
        if k == "model.embed_tokens.weight":
            out["tok_embeddings.weight"] = v
        elif k == "model.norm.weight":
            out["norm.weight"] = v
        elif k == "lm_head.weight":
            out["output.weight"] = v
        else:
            m = re.match(r"^model\.(layers\.\d+\.)(.+)\.weight$", k)
            if m and m.group(2) in _HF_TO_META:
                out[f"{m.group(1)}{_HF_TO_META[m.group(2)]}.weight"] = v
    return out


def num_layers_of(sd, pattern=r"^layers\.(\d+)\."):
    ids = {int(m.group(1)) for k in sd for m in [re.match(pattern, k)] if m}
    return max(ids) + 1 if ids else 0


def llama_to_megatron(meta_sd, n_heads, n_heads_kv=None, source="meta"):
    """Meta-keyed Llama weights -> canonical Megatron dict (``source='hf'``
    applies the rotate-half -> interleaved QKV permutation)."""
    n_heads_kv = n_heads_kv or n_heads
    hidden = meta_sd["tok_embeddings.weight"].shape[1]
    tr = {"final_layernorm.weight": meta_sd["norm.weight"]}
    for i in range(num_layers_of(meta_sd)):
        p = f"layers.{i}"
        qkv = pack_qkv(meta_sd[f"{p}.attention.wq.weight"], meta_sd[f"{p}.attention.wk.weight"],
                       meta_sd[f"{p}.attention.wv.weight"], n_heads, n_heads_kv)
        if source == "hf":
            qkv = permute_qkv(qkv, hidden, n_heads, n_heads_kv)
        tr[f"{p}.attention.query_key_value.weight"] = qkv
        tr[f"{p}.attention.dense.weight"] = meta_sd[f"{p}.attention.wo.weight"]
        tr[f"{p}.input_layernorm.weight"] = meta_sd[f"{p}.attention_norm.weight"]
        tr[f"{p}.post_attention_layernorm.weight"] = meta_sd[f"{p}.ffn_norm.weight"]
        tr[f"{p}.mlp.dense_h_to_4h.weight"] = torch.cat(
            (meta_sd[f"{p}.feed_forward.w3.weight"], meta_sd[f"{p}.feed_forward.w1.weight"]))
        tr[f"{p}.mlp.dense_4h_to_h.weight"] = meta_sd[f"{p}.feed_forward.w2.weight"]
    return {"embedding": {"word_embeddings.weight": meta_sd["tok_embeddings.weight"]},
            "transformer": tr, "lm_head": meta_sd["output.weight"]}


def megatron_to_hf_llama(full, n_heads, n_heads_kv=None, vocab_size=None):
    """Canonical Megatron dict -> HF ``LlamaForCausalLM`` state dict."""
    n_heads_kv = n_heads_kv or n_heads
    tr = full["transformer"]
    emb = full["embedding"]["word_embeddings.weight"]
    hidden = emb.shape[1]
    hd = hidden // n_heads
    v = vocab_size or emb.shape[0]
    out = {"model.embed_tokens.weight": emb[:v], "model.norm.weight": tr["final_layernorm.weight"],
           "lm_head.weight": (full["lm_head"] if "lm_head" in full else emb)[:v]}
    for i in range(num_layers_of(tr)):
        p, q = f"layers.{i}", f"model.layers.{i}"
        qkv = permute_qkv(tr[f"{p}.attention.query_key_value.weight"], hidden, n_heads,
                          n_heads_kv, revert=True)
        wq, wk, wv = unpack_qkv(qkv, n_heads, n_heads_kv, hd)
        up, gate = torch.chunk(tr[f"{p}.mlp.dense_h_to_4h.weight"], 2, dim=0)
        out.update({
            f"{q}.self_attn.q_proj.weight": wq, f"{q}.self_attn.k_proj.weight": wk,
            f"{q}.self_attn.v_proj.weight": wv,
            f"{q}.self_attn.o_proj.weight": tr[f"{p}.attention.dense.weight"],
            f"{q}.mlp.gate_proj.weight": gate.contiguous(), f"{q}.mlp.up_proj.weight": up.contiguous(),
            f"{q}.mlp.down_proj.weight": tr[f"{p}.mlp.dense_4h_to_h.weight"],
            f"{q}.input_layernorm.weight": tr[f"{p}.input_layernorm.weight"],
            f"{q}.post_attention_layernorm.weight": tr[f"{p}.post_attention_layernorm.weight"],
        })
    return out


def llama_args(num_layers, hidden, heads, ffn, kv_heads, version=2, vocab=32000,
               norm_eps=None, seq_length=None):
    """Training args stored in a converted checkpoint (reference weights2megatron.py:186-211)."""
    a = dict(num_layers=num_layers, hidden_size=hidden, num_attention_heads=heads,
             num_attention_heads_kv=kv_heads, ffn_hidden_size=ffn, parallel_attn=False,
             make_vocab_size_divisible_by=1, glu_activation="swiglu",
             padded_vocab_size=vocab, use_rms_norm=True, tie_embed_logits=False,
             tokenizer_type="SentencePieceTokenizer", use_bias=False)
    seq = seq_length or (2048 if version == 1 else 4096)
    a.update(max_position_embeddings=seq, seq_length=seq,
             layernorm_epsilon=norm_eps or (1e-6 if version == 1 else 1e-5))
    return a

"""Tensor/pipeline-parallel split and merge rules for whole-model state dicts.

The canonical *full* form (one process, TP = PP = 1) is the reference's
release layout (``weights2megatron/weights2megatron.py:172-222``)::

    {"embedding":   {"word_embeddings.weight": [v, h], ["position_embeddings.weight"]},
     "transformer": {"layers.<i>.<...>": ..., "final_layernorm.weight": ...},
     ["lm_head": [v, h]]}

TP rules (reference ``tools/checkpoint_loader_megatron.py:211-300`` and
``checkpoint_saver_megatron.py:229-304``):

* vocab-parallel (dim 0): word embeddings, lm_head;
* column-parallel (dim 0): ``query_key_value`` (grouped per KV head, so
  contiguous chunks are whole KV groups as long as ``n_kv % tp == 0``),
  ``dense_h_to_4h`` — for GLU the up and gate halves are chunked separately
  and re-concatenated per rank;
* row-parallel (dim 1): ``attention.dense.weight``, ``dense_4h_to_h.weight``;
* replicated: norms, row-parallel biases, position embeddings.

PP rules: stage ``p`` owns layers ``[p*L/pp, (p+1)*L/pp)`` renumbered from 0;
the embedding lives on the first stage, ``final_layernorm`` and the LM head on
the last (with tied embeddings the last stage keeps a copy of the word
embeddings under ``word_embeddings_for_head``).
"""
import re

import torch

_LAYER = re.compile(r"^layers\.(\d+)\.(.+)$")


def tp_rule(name):
    """-> ("vocab"|"col"|"glu"|"row"|"rep") for a canonical transformer key."""
    if name.endswith(("query_key_value.weight", "query_key_value.bias")):
        return "col"
    if name.endswith(("dense_h_to_4h.weight", "dense_h_to_4h.bias")):
        return "glu_or_col"
    if name.endswith(("attention.dense.weight", "dense_4h_to_h.weight")):
        return "row"
    return "rep"


def _split(t, rule, tp, glu):
    if rule == "glu_or_col":
        rule = "glu" if glu else "col"
    if rule in ("col", "vocab"):
        return list(torch.chunk(t, tp, dim=0))
    if rule == "row":
        return list(torch.chunk(t, tp, dim=1))
    if rule == "glu":
        up, gate = torch.chunk(t, 2, dim=0)
        return [torch.cat((u, g), dim=0) for u, g in zip(torch.chunk(up, tp, 0),
                                                          torch.chunk(gate, tp, 0))]
    return [t] * tp


def _merge(parts, rule, glu):
    if rule == "glu_or_col":
        rule = "glu" if glu else "col"
    if rule in ("col", "vocab"):
        return torch.cat(parts, dim=0)
    if rule == "row":
        return torch.cat(parts, dim=1)
    if rule == "glu":
        ups, gates = zip(*(torch.chunk(p, 2, dim=0) for p in parts))
        return torch.cat(list(ups) + list(gates), dim=0)
    return parts[0]


def pad_vocab(t, padded_rows):
    """Trim, or pad by replicating the last row, a ``[v, h]`` table to
    ``padded_rows`` (reference ``tools/checkpoint_saver_megatron.py:189-216``)."""
    if t.shape[0] == padded_rows:
        return t
    if t.shape[0] > padded_rows:
        return t[:padded_rows].clone()
    pad = t[-1:].expand(padded_rows - t.shape[0], *t.shape[1:])
    return torch.cat((t, pad), dim=0)


def split_full(full, tp, pp, num_layers, glu, tie_embed_logits, padded_vocab=None):
    """Full canonical dict -> ``shards[pp_rank][tp_rank]`` model dicts
    (``{"language_model": ..., ["word_embeddings_for_head": {"weight": ...}]}``)."""
    if num_layers % pp:
        raise ValueError(f"num_layers {num_layers} not divisible by pipeline size {pp}")
    per = num_layers // pp
    emb = dict(full["embedding"])
    if padded_vocab is not None:
        emb["word_embeddings.weight"] = pad_vocab(emb["word_embeddings.weight"], padded_vocab)
    head = full.get("lm_head")
    if head is not None and padded_vocab is not None:
        head = pad_vocab(head, padded_vocab)
    word = _split(emb["word_embeddings.weight"], "vocab", tp, glu)
    heads = _split(head, "vocab", tp, glu) if head is not None else None
    shards = [[{"language_model": {}} for _ in range(tp)] for _ in range(pp)]
    # transformer
    per_key = {}
    for name, t in full["transformer"].items():
        m = _LAYER.match(name)
        if m:
            layer = int(m.group(1))
            stage, local = divmod(layer, per)
            key = f"layers.{local}.{m.group(2)}"
        else:
            stage, key = pp - 1, name
        parts = _split(t, tp_rule(key), tp, glu)
        for r in range(tp):
            per_key.setdefault((stage, r), {})[key] = parts[r]
    for p in range(pp):
        for r in range(tp):
            lm = shards[p][r]["language_model"]
            lm["transformer"] = per_key.get((p, r), {})
            if p == 0:
                e = {k: v for k, v in emb.items() if k != "word_embeddings.weight"}
                e["word_embeddings.weight"] = word[r]
                lm["embedding"] = e
            if p == pp - 1:
                if heads is not None and not tie_embed_logits:
                    lm["lm_head"] = heads[r]
                elif pp > 1 and tie_embed_logits:
                    shards[p][r]["word_embeddings_for_head"] = {"weight": word[r]}
    return shards


def canonical_lm(lm):
    """Normalise a saved ``language_model`` dict (ours or the reference's) to the
    canonical keys: ``transformer``/``attention``/flat ``*.weight`` names."""
    out = {}
    emb = lm.get("embedding", {})
    flat = {}
    for k, v in emb.items():
        if isinstance(v, dict):
            for kk, vv in v.items():
                flat[f"{k}.{kk}"] = vv
        else:
            flat[k] = v
    if flat:
        out["embedding"] = flat
    tr = lm.get("transformer", lm.get("encoder"))
    if tr is not None:
        out["transformer"] = {k.replace(".self_attention.", ".attention."): v
                              for k, v in tr.items()}
    if "lm_head" in lm:
        out["lm_head"] = lm["lm_head"]
    return out


def merge_shards(shards, num_layers, glu):
    """``shards[pp_rank][tp_rank]`` model dicts -> full canonical dict."""
    pp, tp = len(shards), len(shards[0])
    per = num_layers // pp
    full = {"embedding": {}, "transformer": {}}
    lms = [[canonical_lm(shards[p][r]["language_model"]) for r in range(tp)] for p in range(pp)]
    for k in lms[0][0].get("embedding", {}):
        parts = [lms[0][r]["embedding"][k] for r in range(tp)]
        full["embedding"][k] = _merge(parts, "vocab" if k.startswith("word_") else "rep", glu)
    for p in range(pp):
        for k in lms[p][0].get("transformer", {}):
            parts = [lms[p][r]["transformer"][k] for r in range(tp)]
            m = _LAYER.match(k)
            gk = f"layers.{p * per + int(m.group(1))}.{m.group(2)}" if m else k
            full["transformer"][gk] = _merge(parts, tp_rule(k), glu)
    if "lm_head" in lms[-1][0]:
        full["lm_head"] = _merge([lms[-1][r]["lm_head"] for r in range(tp)], "vocab", glu)
    return full

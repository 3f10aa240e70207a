"""Shared helpers for the BERT-style finetuning tasks (reference
``tasks/data_utils.py``): text clean-up and the ``[CLS] a [SEP] b [SEP]``
token/type/padding layout consumed by ``Classification`` / ``MultipleChoice``.
"""
import re

import numpy as np

_WS = re.compile(r"\s+")


def clean_text(text):
    """Newlines -> spaces, collapse whitespace, glue `` . `` onto the previous
    word (three passes, as the reference does, so runs of dots collapse)."""
    text = _WS.sub(" ", text.replace("\n", " "))
    for _ in range(3):
        text = text.replace(" . ", ". ")
    return text


def build_sample(ids, types, paddings, label, unique_id):
    return {"text": np.asarray(ids, dtype=np.int64),
            "types": np.asarray(types, dtype=np.int64),
            "padding_mask": np.asarray(paddings, dtype=np.int64),
            "label": int(label), "uid": int(unique_id)}


def build_tokens_types_paddings_from_ids(a_ids, b_ids, max_seq_length, cls_id, sep_id, pad_id):
    """Layout ``[CLS] a [SEP] (b) ... [SEP] PAD*``.

    Types are 0 for the CLS/a segment and 1 for b.  When the sequence
    reaches ``max_seq_length`` it is cut to ``max_seq_length-1`` and a final
    [SEP] is appended; a trailing [SEP] is also added when b is present.
    Padded positions carry ``pad_id`` for both ids and types (reference
    behaviour) and 0 in the padding mask.
    """
    ids = [cls_id, *a_ids, sep_id]
    types = [0] * len(ids)
    if b_ids is not None:
        ids += list(b_ids)
        types += [1] * len(b_ids)
    trimmed = len(ids) >= max_seq_length
    if trimmed:
        ids, types = ids[:max_seq_length - 1], types[:max_seq_length - 1]
    if b_ids is not None or trimmed:
        ids.append(sep_id)
        types.append(0 if b_ids is None else 1)
    n = len(ids)
    pad = max_seq_length - n
    paddings = [1] * n + [0] * max(pad, 0)
    if pad > 0:
        ids += [pad_id] * pad
        types += [pad_id] * pad
    return ids, types, paddings


def build_tokens_types_paddings_from_text(text_a, text_b, tokenizer, max_seq_length):
    a = tokenizer.tokenize(text_a)
    b = tokenizer.tokenize(text_b) if text_b is not None else None
    return build_tokens_types_paddings_from_ids(a, b, max_seq_length, tokenizer.cls,
                                                tokenizer.sep, tokenizer.pad)

"""Sentence-pair and span-masking sample construction (BERT / T5 / ICT).

Behavioural spec: reference ``megatron/data/dataset_utils.py:95-419``.  Every
random decision is drawn from the caller's ``np.random.RandomState`` in the
same order as the reference, so a sample index produces the same tokens,
masks and labels in both frameworks:

1. ``shuffle`` of the n-gram candidate list,
2. per accepted candidate: the n-gram length (``choice`` over 1..max_ngrams
   with p ~ 1/n, or ``geometric(0.2)`` clipped for span masking),
3. per masked position (BERT style): ``random() < .8`` -> [MASK], else
   ``random() < .5`` -> keep, else ``randint(vocab)``,
4. a second ``shuffle`` of the candidates (used by the permutation option).
"""
import collections

import numpy as np

MaskedLmInstance = collections.namedtuple("MaskedLmInstance", ["index", "label"])


def get_a_and_b_segments(sample, np_rng):
    """Split a multi-sentence sample into segments A and B; swap them half of
    the time (the "random next" label of the sentence-order head)."""
    n = len(sample)
    if n < 2:
        raise AssertionError("make sure each sample has at least two sentences.")
    a_end = np_rng.randint(1, n) if n >= 3 else 1
    tokens_a = [t for sent in sample[:a_end] for t in sent]
    tokens_b = [t for sent in sample[a_end:] for t in sent]
    is_next_random = bool(np_rng.random() < 0.5)
    if is_next_random:
        tokens_a, tokens_b = tokens_b, tokens_a
    return tokens_a, tokens_b, is_next_random


def truncate_segments(tokens_a, tokens_b, len_a, len_b, max_num_tokens, np_rng):
    """Trim the longer segment one token at a time (front or back at random)
    until the pair fits; returns whether anything was cut."""
    if len_a <= 0:
        raise AssertionError("segment A is empty")
    if len_a + len_b <= max_num_tokens:
        return False
    while len_a + len_b > max_num_tokens:
        if len_a > len_b:
            len_a -= 1
            seg = tokens_a
        else:
            len_b -= 1
            seg = tokens_b
        if np_rng.random() < 0.5:
            del seg[0]
        else:
            seg.pop()
    return True


def create_tokens_and_tokentypes(tokens_a, tokens_b, cls_id, sep_id):
    """``[CLS] A [SEP] (B [SEP])`` with token types 0 for A, 1 for B."""
    tokens = [cls_id] + list(tokens_a) + [sep_id]
    types = [0] * len(tokens)
    if tokens_b:
        tokens += list(tokens_b) + [sep_id]
        types += [1] * (len(tokens_b) + 1)
    return tokens, types


def is_start_piece(piece):
    """WordPiece continuation pieces start with '##'."""
    return not piece.startswith("##")


def _flatten(spans):
    return [i for span in spans for i in span]


def create_masked_lm_predictions(tokens, vocab_id_list, vocab_id_to_token_dict, masked_lm_prob,
                                 cls_id, sep_id, mask_id, max_predictions_per_seq, np_rng,
                                 max_ngrams=3, do_whole_word_mask=True, favor_longer_ngram=False,
                                 do_permutation=False, geometric_dist=False,
                                 masking_style="bert"):
    """Whole-word n-gram masking.

    Returns ``(output_tokens, masked_positions, masked_labels, token_boundary,
    masked_spans)`` (the last entry is absent when ``masked_lm_prob == 0``,
    matching the reference's short return).
    """
    # word candidates: lists of positions; '##' pieces join the previous word
    words = []
    boundary = [0] * len(tokens)
    for i, tok in enumerate(tokens):
        if tok == cls_id or tok == sep_id:
            boundary[i] = 1
            continue
        starts = is_start_piece(vocab_id_to_token_dict[tok])
        if do_whole_word_mask and words and not starts:
            words[-1].append(i)
        else:
            words.append([i])
            if starts:
                boundary[i] = 1
    out = list(tokens)
    if masked_lm_prob == 0:
        return out, [], [], boundary

    budget = min(max_predictions_per_seq, max(1, int(round(len(tokens) * masked_lm_prob))))
    ngram_sizes = np.arange(1, max_ngrams + 1, dtype=np.int64)
    pvals = None
    if not geometric_dist:
        pvals = 1.0 / np.arange(1, max_ngrams + 1)
        pvals /= pvals.sum(keepdims=True)
        if favor_longer_ngram:
            pvals = pvals[::-1]
    # candidate c = [words[c:c+1], words[c:c+2], ..., words[c:c+max_ngrams]]
    candidates = [[words[c:c + n] for n in ngram_sizes] for c in range(len(words))]
    np_rng.shuffle(candidates)

    def pick_length(cand):
        if geometric_dist:
            return min(np_rng.geometric(0.2), max_ngrams)
        k = len(cand)
        return np_rng.choice(ngram_sizes[:k], p=pvals[:k] / pvals[:k].sum(keepdims=True))

    def shrink_to_fit(cand, n, used):
        # try the drawn length, then successively shorter ones
        idx = _flatten(cand[n - 1])
        n -= 1
        while used + len(idx) > budget:
            if n == 0:
                break
            idx = _flatten(cand[n - 1])
            n -= 1
        return idx

    masked, spans = [], []
    covered = set()
    for cand in candidates:
        if len(masked) >= budget:
            break
        if not cand:
            continue
        idx = shrink_to_fit(cand, pick_length(cand), len(masked))
        if len(masked) + len(idx) > budget:
            continue
        if any(i in covered for i in idx):
            continue
        for i in idx:
            covered.add(i)
            if masking_style == "bert":
                if np_rng.random() < 0.8:
                    new = mask_id
                elif np_rng.random() < 0.5:
                    new = tokens[i]
                else:
                    new = vocab_id_list[np_rng.randint(0, len(vocab_id_list))]
            elif masking_style == "t5":
                new = mask_id
            else:
                raise ValueError("invalid value of masking style")
            out[i] = new
            masked.append(MaskedLmInstance(index=i, label=tokens[i]))
        spans.append(MaskedLmInstance(index=idx, label=[tokens[i] for i in idx]))
    if len(masked) > budget:
        raise AssertionError("masked more tokens than the budget")
    np_rng.shuffle(candidates)

    if do_permutation:
        chosen = set()
        for cand in candidates:
            if len(chosen) >= budget:
                break
            if not cand:
                continue
            # the reference draws this length from the *global* numpy RNG
            k = len(cand)
            n = np.random.choice(ngram_sizes[:k], p=pvals[:k] / pvals[:k].sum(keepdims=True))
            idx = shrink_to_fit(cand, n, len(chosen))
            if len(chosen) + len(idx) > budget:
                continue
            if any(i in covered or i in chosen for i in idx):
                continue
            chosen.update(idx)
        src = sorted(chosen)
        dst = list(src)
        np_rng.shuffle(dst)
        before = list(out)
        for s, t in zip(src, dst):
            out[s] = before[t]
            masked.append(MaskedLmInstance(index=s, label=before[s]))

    masked.sort(key=lambda m: m.index)
    spans.sort(key=lambda m: m.index[0])
    return (out, [m.index for m in masked], [m.label for m in masked], boundary, spans)


def pad_and_convert_to_numpy(tokens, tokentypes, masked_positions, masked_labels, pad_id,
                             max_seq_length):
    """BERT sample arrays: tokens, types, labels (-1 = unmasked), padding mask,
    loss mask — all int64 ``[max_seq_length]``."""
    n = len(tokens)
    pad = max_seq_length - n
    if pad < 0 or len(tokentypes) != n or len(masked_positions) != len(masked_labels):
        raise AssertionError("inconsistent sample")
    tokens_np = np.array(list(tokens) + [pad_id] * pad, dtype=np.int64)
    types_np = np.array(list(tokentypes) + [pad_id] * pad, dtype=np.int64)
    padding_mask = np.array([1] * n + [0] * pad, dtype=np.int64)
    labels = np.full(max_seq_length, -1, dtype=np.int64)
    loss_mask = np.zeros(max_seq_length, dtype=np.int64)
    for pos, lab in zip(masked_positions, masked_labels):
        if pos >= n:
            raise AssertionError("masked position beyond the sample")
        labels[pos] = lab
        loss_mask[pos] = 1
    return tokens_np, types_np, labels, padding_mask, loss_mask

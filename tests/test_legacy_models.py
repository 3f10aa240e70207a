"""Legacy model families (BERT, T5, ICT bi-encoder, classification heads) and
their sentence-level data pipeline, on CPU/gloo.

* The native sample maps are checked against a pure-Python transcription of
  the reference algorithm (megatron/data/helpers.cpp build_mapping /
  build_blocks_mapping) driven by the same Mersenne twisters, so cached
  ``*_indexmap_*.npy`` files are interchangeable.
* Masking: budget, labels and whole-word grouping invariants.
* Each family trains a few steps through ``pretrain_*.py``'s forward/loss
  functions; BERT and T5 losses are identical at TP=1 and TP=2 (parity of the
  vocab-parallel heads).  No HF/Meta checkpoints exist for these legacy
  models in this environment: numerical parity with an external
  implementation is unpinned.
"""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from epfl_megatron_amd.data import helpers  # noqa: E402
from epfl_megatron_amd.data import indexed_dataset as idx_ds  # noqa: E402
from epfl_megatron_amd.data.masking import create_masked_lm_predictions  # noqa: E402


# ---------------------------------------------------------------- RNG oracles
class _MT19937_64:
    """std::mt19937_64 (for the oracle of the reference's shuffle)."""

    def __init__(self, seed):
        self.mt = [0] * 312
        self.mt[0] = seed & 0xFFFFFFFFFFFFFFFF
        for i in range(1, 312):
            self.mt[i] = (6364136223846793005 * (self.mt[i - 1] ^ (self.mt[i - 1] >> 62)) + i) \
                & 0xFFFFFFFFFFFFFFFF
        self.i = 312

    def __call__(self):
        if self.i >= 312:
            for k in range(312):
                x = (self.mt[k] & 0xFFFFFFFF80000000) | (self.mt[(k + 1) % 312] & 0x7FFFFFFF)
                xa = x >> 1
                if x & 1:
                    xa ^= 0xB5026F5AA96619E9
                self.mt[k] = self.mt[(k + 156) % 312] ^ xa
            self.i = 0
        y = self.mt[self.i]
        self.i += 1
        y ^= (y >> 29) & 0x5555555555555555
        y ^= (y << 17) & 0x71D67FFFEDA60000
        y ^= (y << 37) & 0xFFF7EEE000000000
        y ^= y >> 43
        return y & 0xFFFFFFFFFFFFFFFF


class _MT19937:
    """std::mt19937(seed) via numpy's legacy generator (same init_genrand)."""

    def __init__(self, seed):
        self.rs = np.random.RandomState(seed)

    def __call__(self):
        return int(self.rs.randint(0, 2 ** 32, dtype=np.uint64))


def _oracle_mapping(docs, sizes, num_epochs, max_samples, max_len, short_prob, seed, min_sent):
    ratio = int(round(1.0 / short_prob)) if short_prob > 0 else 0
    g = _MT19937(seed)

    def target():
        if ratio == 0:
            return max_len
        r = g()
        return 2 + r % (max_len - 1) if r % ratio == 0 else max_len

    rows = []
    for _ in range(num_epochs):
        if len(rows) >= max_samples:
            break
        for d in range(len(docs) - 1):
            first, last = docs[d], docs[d + 1]
            remain = last - first
            long_ = remain > 1 and any(sizes[first:last] > 512)
            if remain < min_sent or long_:
                continue
            start, ln, ns, tgt = first, 0, 0, target()
            for s in range(first, last):
                ln += sizes[s]
                ns += 1
                remain -= 1
                if (ln >= tgt and remain > 1 and ns >= min_sent) or remain == 0:
                    rows.append([start, s + 1, tgt])
                    start, ln, ns, tgt = s + 1, 0, 0, target()
    g64 = _MT19937_64(seed + 1)
    for i in range(len(rows) - 1, 0, -1):
        j = g64() % (i + 1)
        rows[i], rows[j] = rows[j], rows[i]
    return np.array(rows, dtype=np.uint32).reshape(-1, 3)


def _sentence_corpus(n_docs=40, seed=0, vocab=200, long_every=0):
    rng = np.random.default_rng(seed)
    docs, sizes = [0], []
    for d in range(n_docs):
        n = int(rng.integers(0, 7))
        for _ in range(n):
            sizes.append(int(rng.integers(1, 30)) if not (long_every and d % long_every == 0)
                         else 600)
        docs.append(len(sizes))
    return np.array(docs, dtype=np.int64), np.array(sizes, dtype=np.int32)


@pytest.mark.parametrize("short_prob,min_sent", [(0.1, 2), (0.0, 1), (0.5, 2)])
def test_sentence_mapping_matches_reference_algorithm(short_prob, min_sent):
    docs, sizes = _sentence_corpus(60, seed=4, long_every=13)
    got = helpers.build_mapping(docs, sizes, 3, 10 ** 9, 40, short_prob, 1234, False, min_sent)
    want = _oracle_mapping(docs, sizes, 3, 10 ** 9, 40, short_prob, 1234, min_sent)
    assert got.dtype == np.uint32 and got.shape == want.shape
    np.testing.assert_array_equal(got, want)


def test_block_mapping_invariants():
    docs, sizes = _sentence_corpus(50, seed=5)
    titles = np.random.default_rng(1).integers(1, 5, size=50).astype(np.int32)
    m = helpers.build_blocks_mapping(docs, sizes, titles, 1, 10 ** 9, 32, 7, False, False)
    assert m.shape[1] == 4
    ids = sorted(int(b) for b in m[:, 3])
    assert ids == list(range(len(ids)))  # block ids unique and dense per epoch
    for start, end, doc, _ in m:
        assert docs[doc] <= start < end <= docs[doc + 1]


def test_masked_lm_invariants():
    vocab = {i: (f"##p{i}" if i % 4 == 3 else f"w{i}") for i in range(10, 200)}
    vocab.update({1: "[CLS]", 2: "[SEP]", 3: "[MASK]"})
    rng = np.random.RandomState(3)
    toks = [1] + list(rng.randint(10, 200, size=60)) + [2]
    out, pos, labels, boundary, spans = create_masked_lm_predictions(
        toks, list(vocab.keys()), vocab, 0.15, 1, 2, 3, 0.15 * 62, np.random.RandomState(9))
    assert 0 < len(pos) <= round(0.15 * 62) + 1
    assert pos == sorted(pos) and all(toks[p] == lab for p, lab in zip(pos, labels))
    assert 0 not in pos and len(toks) - 1 not in pos  # [CLS]/[SEP] never masked
    changed = [i for i in range(len(toks)) if out[i] != toks[i]]
    assert set(changed) <= set(pos)
    # whole-word: a masked '##' piece implies its word start is masked too
    for p in pos:
        if vocab[toks[p]].startswith("##") and p > 1 and not vocab[toks[p - 1]].startswith("##"):
            assert p - 1 in pos
    # deterministic for a given RNG seed
    again = create_masked_lm_predictions(toks, list(vocab.keys()), vocab, 0.15, 1, 2, 3,
                                         0.15 * 62, np.random.RandomState(9))
    assert again[0] == out and again[1] == pos


# ---------------------------------------------------------------- training
WORDS = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + [f"w{i}" for i in range(100)] + \
    [f"##s{i}" for i in range(20)]


def _write_corpus(tmp, name="corpus", n_docs=60, seed=0):
    """Sentence-split corpus (doc_idx with several sentences per document)."""
    rng = np.random.default_rng(seed)
    prefix = str(tmp / name)
    b = idx_ds.MMapIndexedDatasetBuilder(prefix + ".bin", dtype=np.uint16)
    for _ in range(n_docs):
        for _ in range(int(rng.integers(2, 6))):
            b.add_item(torch.tensor(rng.integers(5, len(WORDS), size=int(rng.integers(3, 12)))))
        b.end_document()
    b.finalize(prefix + ".idx")
    return prefix


def _vocab_file(tmp):
    p = tmp / "vocab.txt"
    p.write_text("\n".join(WORDS) + "\n")
    return str(p)


BERT_TINY = ["--num_layers", "2", "--hidden_size", "64", "--num_attention_heads", "4",
             "--seq_length", "32", "--max_position_embeddings", "64", "--micro_batch_size", "2",
             "--global_batch_size", "4", "--hidden_dropout", "0.0", "--attention_dropout", "0.0",
             "--lr", "1e-3", "--train_iters", "3", "--seed", "1234", "--log_interval", "1000",
             "--eval_iters", "0", "--eval_interval", "1000", "--use_cpu_initialization",
             "--tokenizer_type", "BertWordPieceLowerCase", "--make_vocab_size_divisible_by", "8",
             "--split", "10,0,0", "--data_impl", "mmap", "--clip_grad", "1.0", "--use_bias",
             "--distributed_backend", "gloo", "--num_workers", "0"]


def _run_steps(module_name, argv, steps=3):
    import importlib
    mod = importlib.import_module(module_name)
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.initialize import initialize_megatron
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.training import (_setup_model_and_optimizer,
                                            build_train_valid_test_data_iterators, train_step)
    initialize_megatron(None, {}, args_list=argv)
    args = get_args()
    provider = getattr(mod, "model_provider", None) or mod.pretrain_ict_model_provider
    mtype = ModelType.encoder_and_decoder if module_name == "pretrain_t5" \
        else ModelType.encoder_or_decoder
    chunks, opt, sched = _setup_model_and_optimizer(provider, mtype, args=args)
    it, _, _ = build_train_valid_test_data_iterators(mod.train_valid_test_datasets_provider,
                                                     args)
    losses = []
    for _ in range(steps):
        out = train_step(mod.forward_step, it, chunks, opt, sched, args)
        args.consumed_train_samples += args.global_batch_size
        losses.append({k: float(v) for k, v in out[0].items()})
    return losses


def _bert_worker(rank, world, argv):
    return _run_steps("pretrain_bert", argv)


def _t5_worker(rank, world, argv):
    return _run_steps("pretrain_t5", argv)


def _ict_worker(rank, world, argv):
    return _run_steps("pretrain_ict", argv)


@pytest.mark.parametrize("binary_head", [True, False])
def test_bert_pretrain_tp_parity(tmp_path, binary_head):
    from dist_utils import run_dist
    argv = BERT_TINY + ["--data_path", _write_corpus(tmp_path), "--vocab_file",
                        _vocab_file(tmp_path)]
    if not binary_head:
        argv += ["--bert_no_binary_head"]
    one = run_dist(_bert_worker, 1, argv)[0]
    two = run_dist(_bert_worker, 2, argv + ["--tensor_model_parallel_size", "2"])
    assert all(np.isfinite(v) for step in one for v in step.values())
    assert ("sop loss" in one[0]) == binary_head
    for a, b in zip(one, two[0]):
        for k in a:
            assert abs(a[k] - b[k]) < 2e-4 * max(1.0, abs(a[k])), (k, a, b)


def test_t5_pretrain_tp_parity(tmp_path):
    from dist_utils import run_dist
    argv = [a for a in BERT_TINY]
    i = argv.index("--seq_length")
    argv[i:i + 2] = ["--encoder_seq_length", "32"]
    argv += ["--decoder_seq_length", "16", "--vocab_extra_ids", "10", "--data_path",
             _write_corpus(tmp_path), "--vocab_file", _vocab_file(tmp_path)]
    one = run_dist(_t5_worker, 1, argv)[0]
    two = run_dist(_t5_worker, 2, argv + ["--tensor_model_parallel_size", "2"])
    assert all(np.isfinite(s["lm loss"]) for s in one)
    for a, b in zip(one, two[0]):
        assert abs(a["lm loss"] - b["lm loss"]) < 2e-4 * max(1.0, a["lm loss"]), (a, b)


def test_ict_pretrain_dp2(tmp_path):
    from dist_utils import run_dist
    blocks = _write_corpus(tmp_path, "blocks", n_docs=60, seed=1)
    rng = np.random.default_rng(2)
    b = idx_ds.MMapIndexedDatasetBuilder(str(tmp_path / "titles.bin"), dtype=np.uint16)
    for _ in range(60):
        b.add_item(torch.tensor(rng.integers(5, len(WORDS), size=3)))
        b.end_document()
    b.finalize(str(tmp_path / "titles.idx"))
    argv = BERT_TINY + ["--data_path", blocks, "--titles_data_path", str(tmp_path / "titles"),
                        "--vocab_file", _vocab_file(tmp_path), "--query_in_block_prob", "0.5",
                        "--retriever_report_topk_accuracies", "1", "2",
                        "--biencoder_projection_dim", "16"]
    res = run_dist(_ict_worker, 2, argv)
    assert res[0] == res[1]  # DP ranks see the same gathered score matrix
    assert all(np.isfinite(s["loss"]) and 0.0 <= s["top1_acc"] <= 100.0 for s in res[0])


def _heads_worker(rank, world, argv):
    from epfl_megatron_amd.initialize import initialize_megatron
    from epfl_megatron_amd.models import Classification, MultipleChoice
    initialize_megatron(None, {}, args_list=argv)
    torch.manual_seed(0)
    cls = Classification(num_classes=3)
    ids = torch.randint(5, 100, (4, 16))
    mask = torch.ones(4, 16, dtype=torch.long)
    mask[:, 12:] = 0
    logits = cls(ids, mask, tokentype_ids=torch.zeros_like(ids))
    mc = MultipleChoice()
    mlog = mc(ids.view(2, 2, 16), mask.view(2, 2, 16), tokentype_ids=torch.zeros(2, 2, 16,
                                                                                 dtype=torch.long))
    (logits.sum() + mlog.sum()).backward()
    sd = cls.state_dict_for_save_checkpoint()
    return (tuple(logits.shape), tuple(mlog.shape), sorted(sd.keys()))


def test_classification_and_multiple_choice_heads(tmp_path):
    from dist_utils import run_dist
    argv = BERT_TINY + ["--vocab_file", _vocab_file(tmp_path)]
    out = run_dist(_heads_worker, 1, argv)[0]
    assert out == ((4, 3), (2, 2), ["classification_head", "language_model"])


def _t5_pp_worker(rank, world, argv, steps=3):
    """T5 steps with every weight filled from its global name (same values at
    any PP split), so PP=2 with a split rank must reproduce PP=1."""
    import importlib
    mod = importlib.import_module("pretrain_t5")
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.initialize import initialize_megatron
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.optim import get_megatron_optimizer
    from epfl_megatron_amd.parallel import state
    from epfl_megatron_amd.training import (get_model, _get_optimizer_param_scheduler,
                                            build_train_valid_test_data_iterators, train_step)
    from test_parallel_equivalence import _deterministic_init
    initialize_megatron(None, {}, args_list=argv)
    args = get_args()
    model = get_model(mod.model_provider, ModelType.encoder_and_decoder)
    _deterministic_init(model, args)
    opt = get_megatron_optimizer(model)
    sched = _get_optimizer_param_scheduler(opt)
    args.iteration = 0
    it, _, _ = build_train_valid_test_data_iterators(mod.train_valid_test_datasets_provider, args)
    losses = []
    for _ in range(steps):
        out = train_step(mod.forward_step, it, model, opt, sched, args)
        args.consumed_train_samples += args.global_batch_size
        if out[0]:
            losses.append((float(out[0]["lm loss"]), float(out[2])))
    return losses if state.is_pipeline_last_stage(ignore_virtual=True) else None


def test_t5_pipeline_split_rank(tmp_path):
    """Encoder on stage 0, decoder on stage 1 (--pipeline_model_parallel_split_rank,
    reference schedules.py:505-535, parallel_state.py:367-403): shared word
    embeddings summed over the embedding group {0, 1}, position embeddings over
    the position-embedding group, losses equal to the single-stage run."""
    from dist_utils import run_dist
    argv = [a for a in BERT_TINY]
    i = argv.index("--seq_length")
    argv[i:i + 2] = ["--encoder_seq_length", "32"]
    argv += ["--decoder_seq_length", "16", "--vocab_extra_ids", "10", "--data_path",
             _write_corpus(tmp_path), "--vocab_file", _vocab_file(tmp_path),
             "--micro_batch_size", "1"]
    one = [r for r in run_dist(_t5_pp_worker, 1, argv) if r][0]
    two = [r for r in run_dist(_t5_pp_worker, 2, argv + [
        "--pipeline_model_parallel_size", "2", "--pipeline_model_parallel_split_rank", "1"])
        if r][0]
    assert len(one) == len(two) == 3
    for (l0, g0), (l1, g1) in zip(one, two):
        assert abs(l0 - l1) < 2e-5 * max(1.0, abs(l0)), (one, two)
        assert abs(g0 - g1) < 1e-4 * max(1.0, abs(g0)), (one, two)

"""Data pipeline: indexed corpora, index maps, blending, preprocess/merge tools.

Mirrors the intent of the reference's data tests (``megatron/data/test``) on
CPU, plus byte-level checks of the on-disk format.
"""
import json
import os
import struct
import subprocess
import sys

import numpy as np
import pytest
import torch

from epfl_megatron_amd.data import indexed_dataset as idx_ds
from epfl_megatron_amd.data import helpers
from epfl_megatron_amd.data.dataset_utils import (get_train_valid_test_split_,
                                                  get_datasets_weights_and_num_samples)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _docs(n=37, seed=0, vocab=1000):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, vocab, size=int(rng.integers(1, 40))) for _ in range(n)]


def _write_mmap(prefix, docs, dtype=np.uint16):
    b = idx_ds.MMapIndexedDatasetBuilder(prefix + ".bin", dtype=dtype)
    for d in docs:
        b.add_item(torch.tensor(d))
        b.end_document()
    b.finalize(prefix + ".idx")


def test_mmap_roundtrip_and_header(tmp_path):
    docs = _docs()
    p = str(tmp_path / "c")
    _write_mmap(p, docs)
    raw = open(p + ".idx", "rb").read()
    assert raw[:9] == b"MMIDIDX\x00\x00"
    assert struct.unpack_from("<Q", raw, 9)[0] == 1
    assert raw[17] == 8  # uint16
    n, ndoc = struct.unpack_from("<QQ", raw, 18)
    assert n == len(docs) and ndoc == len(docs) + 1
    sizes = np.frombuffer(raw, np.int32, n, 34)
    ptrs = np.frombuffer(raw, np.int64, n, 34 + 4 * n)
    assert sizes.tolist() == [len(d) for d in docs]
    assert ptrs.tolist() == (np.cumsum([0] + [2 * len(d) for d in docs[:-1]])).tolist()
    assert os.path.getsize(p + ".bin") == 2 * sum(len(d) for d in docs)
    ds = idx_ds.make_dataset(p, "infer", skip_warmup=True)
    assert isinstance(ds, idx_ds.MMapIndexedDataset) and len(ds) == len(docs)
    for i, d in enumerate(docs):
        np.testing.assert_array_equal(ds[i], d)
    np.testing.assert_array_equal(ds.get(3, offset=1, length=1), docs[3][1:2])
    for a, d in zip(ds[2:6], docs[2:6]):
        np.testing.assert_array_equal(a, d)
    assert ds.doc_idx.tolist() == list(range(len(docs) + 1))


def test_legacy_roundtrip(tmp_path):
    docs = _docs(9, seed=1)
    p = str(tmp_path / "leg")
    b = idx_ds.make_builder(p + ".bin", "cached")
    for d in docs:
        b.add_item(torch.tensor(d))
        b.end_document()
    b.finalize(p + ".idx")
    assert idx_ds.infer_dataset_impl(p) == "cached"
    for impl in ("lazy", "cached"):
        ds = idx_ds.make_dataset(p, impl)
        if impl == "cached":
            ds.prefetch(range(len(docs)))
        for i, d in enumerate(docs):
            np.testing.assert_array_equal(ds[i], d)


def test_merge_tool(tmp_path):
    d1, d2 = _docs(5, 2), _docs(7, 3)
    src = tmp_path / "parts"
    src.mkdir()
    _write_mmap(str(src / "a"), d1)
    _write_mmap(str(src / "b"), d2)
    out = str(tmp_path / "merged")
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "merge_datasets.py"),
                           "--input", str(src), "--output_prefix", out])
    ds = idx_ds.MMapIndexedDataset(out, skip_warmup=True)
    assert len(ds) == 12
    for i, d in enumerate(d1 + d2):
        np.testing.assert_array_equal(ds[i], d)
    assert ds.doc_idx.tolist() == list(range(13))


def _py_sample_idx(sizes, doc_idx, seq, epochs, tpe):
    n = (epochs * tpe - 1) // seq
    out = np.zeros((n + 1, 2), np.int32)
    pos, off = 0, 0
    for s in range(1, n + 1):
        need = seq + 1
        while need:
            avail = sizes[doc_idx[pos]] - off
            if avail >= need:
                off += need - 1
                need = 0
            else:
                need -= avail
                pos += 1
                off = 0
        out[s] = (pos, off)
    return out


def test_sample_idx_native_matches_python():
    rng = np.random.default_rng(5)
    sizes = rng.integers(1, 50, size=100).astype(np.int32)
    doc_idx = np.tile(np.arange(100, dtype=np.int32), 3)
    rng.shuffle(doc_idx)
    tpe = int(sizes.sum())
    for seq in (7, 16, 64):
        np.testing.assert_array_equal(helpers.build_sample_idx(sizes, doc_idx, seq, 3, tpe),
                                      _py_sample_idx(sizes, doc_idx, seq, 3, tpe))


def test_blending_indices_track_weights():
    w = np.array([0.5, 0.3, 0.2])
    which = np.zeros(1000, np.uint8)
    within = np.zeros(1000, np.int64)
    helpers.build_blending_indices(which, within, w, 3, 1000, False)
    counts = np.bincount(which, minlength=3)
    assert np.abs(counts / 1000 - w).max() < 0.01
    for d in range(3):  # samples of each component are consumed in order
        assert within[which == d].tolist() == list(range(counts[d]))


def test_split_and_weights():
    assert get_train_valid_test_split_("969, 30, 1", 1000) == [0, 969, 999, 1000]
    assert get_train_valid_test_split_("80/20", 10) == [0, 8, 10, 10]
    assert get_train_valid_test_split_("1", 7) == [0, 7, 7, 7]
    pre, w, n = get_datasets_weights_and_num_samples(["3", "a", "1", "b"], [100, 10, 0])
    assert pre == ["a", "b"] and w == [0.75, 0.25]
    assert n == [[76, 8, 0], [26, 3, 0]]


def test_gpt_dataset_windows_and_cache(tmp_path):
    from epfl_megatron_amd.data.gpt_dataset import GPTDataset, _num_epochs
    docs = _docs(40, seed=7)
    p = str(tmp_path / "corpus")
    _write_mmap(p, docs)
    ds = idx_ds.MMapIndexedDataset(p, skip_warmup=True)
    seq = 16
    gd = GPTDataset("train", p, np.arange(40, dtype=np.int32), ds, 150, seq, 1234)
    assert len(gd) >= 150
    stream = np.concatenate([docs[i] for i in gd.doc_idx])
    for k in range(len(gd)):
        s = int(gd.shuffle_idx[k])
        want = stream[s * seq: s * seq + seq + 1]
        np.testing.assert_array_equal(gd[k]["text"], want)
    batch = gd.__getitems__([0, 5, 9])
    np.testing.assert_array_equal(batch[1]["text"], gd[5]["text"])
    # python fallback == native
    gd._native = False
    np.testing.assert_array_equal(gd[3]["text"], gd.__getitems__([3])[0]["text"])
    files = sorted(f for f in os.listdir(tmp_path) if "indexmap" in f)
    assert files == [f"corpus_train_indexmap_150ns_16sl_1234s_{k}_idx.npy"
                     for k in ("doc", "sample", "shuffle")]
    # cached maps are reused (same arrays on rebuild)
    gd2 = GPTDataset("train", p, np.arange(40, dtype=np.int32), ds, 150, seq, 1234)
    np.testing.assert_array_equal(gd2.shuffle_idx, gd.shuffle_idx)
    tpe = sum(len(d) for d in docs)
    e = _num_epochs(tpe, seq, 150)
    assert (e * tpe - 1) // seq >= 150 and ((e - 1) * tpe - 1) // seq < 150


def test_gpt_dataset_index_maps_match_reference_algorithm(tmp_path):
    """doc/shuffle maps follow the reference RNG call order (cache interchange)."""
    from epfl_megatron_amd.data.gpt_dataset import GPTDataset
    docs = _docs(30, seed=11)
    p = str(tmp_path / "c2")
    _write_mmap(p, docs)
    ds = idx_ds.MMapIndexedDataset(p, skip_warmup=True)
    seq, n, seed = 8, 100, 42
    gd = GPTDataset("valid", p, np.arange(30, dtype=np.int32), ds, n, seq, seed)
    tpe = sum(len(d) for d in docs)
    epochs = len(gd.doc_idx) // 30
    rng = np.random.RandomState(seed=seed)
    from_full = ((epochs - 1) * tpe - 1) // seq
    per_epoch = (tpe - 1) // seq
    separate = epochs > 1 and (n - from_full) < int(0.8 * per_epoch)
    if separate:
        a = np.mgrid[0:epochs - 1, 0:30][1].reshape(-1).astype(np.int32)
        rng.shuffle(a)
        b = np.arange(30, dtype=np.int32)
        rng.shuffle(b)
        want_doc = np.concatenate([a, b])
    else:
        want_doc = np.mgrid[0:epochs, 0:30][1].reshape(-1).astype(np.int32)
        rng.shuffle(want_doc)
    np.testing.assert_array_equal(gd.doc_idx, want_doc)
    total = gd.sample_idx.shape[0] - 1
    first = from_full if separate else total
    sh = np.arange(first, dtype=np.uint32)
    rng.shuffle(sh)
    if first != total:
        last = np.arange(first, total, dtype=np.uint32)
        rng.shuffle(last)
        sh = np.concatenate([sh, last])
    np.testing.assert_array_equal(gd.shuffle_idx, sh)


def test_build_train_valid_test_blend(tmp_path):
    from epfl_megatron_amd.data.gpt_dataset import build_train_valid_test_datasets
    pa, pb = str(tmp_path / "a"), str(tmp_path / "b")
    _write_mmap(pa, _docs(50, 1))
    _write_mmap(pb, _docs(50, 2))
    tr, va, te = build_train_valid_test_datasets(["0.7", pa, "0.3", pb], "mmap", "8,2,0",
                                                 [64, 8, 0], 8, 1, True)
    assert te is None and len(tr) >= 64 and len(va) >= 8
    assert tr[0]["text"].shape == (9,)
    tr, va, te = build_train_valid_test_datasets(None, "mmap", "", [16, 4, 0], 8, 1, True,
                                                 train_data_prefix=[pa], valid_data_prefix=[pb])
    assert len(tr) >= 16 and len(va) >= 4 and te is None


def _run_preprocess(tmp_path, extra, lines):
    inp = tmp_path / "in.jsonl"
    with open(inp, "w") as f:
        for line in lines:
            f.write(json.dumps(line) + "\n")
    out = str(tmp_path / "out")
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "preprocess_data.py"),
                           "--input", str(inp), "--output_prefix", out, "--chunk_size", "2"]
                          + extra, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return out


@pytest.mark.parametrize("workers", ["1", "2"])
def test_preprocess_null_tokenizer(tmp_path, workers):
    lines = [{"text": " ".join(str(i) for i in range(k, k + 5))} for k in range(0, 50, 5)]
    out = _run_preprocess(tmp_path, ["--tokenizer_type", "NullTokenizer", "--workers", workers,
                                     "--append_eod", "--synthetic_vocab_size", "100"], lines)
    ds = idx_ds.make_dataset(out + "_text_document", "infer")
    assert len(ds) == 10 and ds.dtype == np.uint16
    for i in range(10):
        assert ds[i].tolist() == list(range(5 * i, 5 * i + 5)) + [99]


def test_preprocess_sentencepiece_split_sentences(tmp_path):
    spm = pytest.importorskip("sentencepiece")
    text = ("The quick brown fox jumps over the lazy dog. " * 20 +
            "Pack my box with five dozen liquor jugs! How vexingly quick daft zebras jump? ") * 5
    corpus = tmp_path / "sp.txt"
    corpus.write_text("\n".join(text.split(". ")))
    spm.SentencePieceTrainer.train(input=str(corpus), model_prefix=str(tmp_path / "sp"),
                                   vocab_size=60, model_type="bpe",
                                   minloglevel=2)
    model = str(tmp_path / "sp.model")
    lines = [{"text": "Pack my box. The quick fox! Lazy dog?"}, {"text": "How quick"}]
    out = _run_preprocess(tmp_path, ["--tokenizer_type", "SentencePieceTokenizer",
                                     "--vocab_file", model, "--workers", "1",
                                     "--split_sentences", "--append_eod"], lines)
    ds = idx_ds.make_dataset(out + "_text_sentence", "mmap")
    assert len(ds) == 4  # 3 sentences + 1
    assert ds.doc_idx.tolist() == [0, 3, 4]
    from epfl_megatron_amd.tokenizer.tokenizer import SentencePieceTokenizer
    tok = SentencePieceTokenizer(model)
    assert ds[2][-1] == tok.eod and ds[3][-1] == tok.eod
    assert tok.detokenize(ds[0].tolist()).startswith("Pack my box")


def _train_on_corpus(rank, world, argv):
    import finetune
    from dist_utils import init_framework
    init_framework(argv, finetune.extra_args)
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.training import pretrain
    args = get_args()
    pretrain(args, finetune.train_valid_test_datasets_provider, finetune.model_provider,
             ModelType.encoder_or_decoder, finetune.forward_step)
    return args.consumed_train_samples


def test_finetune_on_indexed_corpus_tp2_dp2(tmp_path):
    from dist_utils import run_dist, TINY_LLAMA
    p = str(tmp_path / "corpus")
    _write_mmap(p, _docs(200, seed=3, vocab=240))
    argv = [a for a in TINY_LLAMA if a != "--synthetic_data"]
    argv += ["--data_path", p, "--split", "9,1,0", "--data_impl", "mmap",
             "--tensor_model_parallel_size", "2", "--micro_batch_size", "1",
             "--global_batch_size", "4", "--eval_interval", "2", "--eval_iters", "1"]
    res = run_dist(_train_on_corpus, 4, argv)
    assert res == [16] * 4
    assert any("indexmap" in f for f in os.listdir(tmp_path))

"""Tokenizers (reference megatron/tokenizer/tokenizer.py): special-token ids,
round trips, vocab padding.  Vocab files are generated in the test (no
downloads)."""
import argparse
import json

import pytest

from epfl_megatron_amd.tokenizer.tokenizer import (build_tokenizer, vocab_size_with_padding,
                                                   NullTokenizer)


def _args(**kw):
    base = dict(rank=1, tokenizer_type=None, vocab_file=None, merge_file=None,
                vocab_extra_ids=0, vocab_extra_ids_list=None, new_tokens=True,
                tokenizer_model=None, make_vocab_size_divisible_by=128,
                tensor_model_parallel_size=1, synthetic_vocab_size=1000)
    base.update(kw)
    return argparse.Namespace(**base)


def test_vocab_padding():
    a = _args(make_vocab_size_divisible_by=128, tensor_model_parallel_size=4)
    assert vocab_size_with_padding(50257, a) == 50688
    assert vocab_size_with_padding(512, a) == 512
    a = _args(make_vocab_size_divisible_by=1, tensor_model_parallel_size=1)
    assert vocab_size_with_padding(32000, a) == 32000


def test_null_tokenizer():
    a = _args(tokenizer_type="NullTokenizer", synthetic_vocab_size=100)
    t = build_tokenizer(a)
    assert isinstance(t, NullTokenizer) and t.vocab_size == 100 and t.eod == 99
    assert t.tokenize("1 2 3") == [1, 2, 3] and t.detokenize([4, 5]) == "4 5"
    assert a.padded_vocab_size == 128


@pytest.fixture(scope="module")
def spm_model(tmp_path_factory):
    spm = pytest.importorskip("sentencepiece")
    d = tmp_path_factory.mktemp("spm")
    text = "\n".join(["the quick brown fox jumps over the lazy dog",
                      "pack my box with five dozen liquor jugs",
                      "how vexingly quick daft zebras jump"] * 30)
    (d / "c.txt").write_text(text)
    spm.SentencePieceTrainer.train(input=str(d / "c.txt"), model_prefix=str(d / "m"),
                                   vocab_size=64, model_type="bpe", minloglevel=2)
    return str(d / "m.model")


def test_sentencepiece_special_tokens(spm_model):
    import sentencepiece as spm
    sp = spm.SentencePieceProcessor(model_file=spm_model)
    n = len(sp)
    a = _args(tokenizer_type="SentencePieceTokenizer", vocab_file=spm_model,
              vocab_extra_ids=2, vocab_extra_ids_list="<a>,<b>")
    t = build_tokenizer(a)
    # new tokens appended in the reference order: CLS SEP EOD MASK PAD, then extras
    assert (t.cls, t.sep, t.eod, t.mask) == (n, n + 1, n + 2, n + 3)
    assert t.pad == n + 4  # the model has no pad piece -> "<PAD>"
    assert t.bos == sp.bos_id() and t.eos == sp.eos_id()
    assert t.vocab["<extra_id_0>"] == n + 5 and t.vocab["<b>"] == n + 8
    assert t.vocab_size == n + 9
    ids = t.tokenize("the quick fox")
    assert t.detokenize(ids) == "the quick fox"
    # special tokens inside text are recognised as single ids
    ids = t.tokenize("the<EOD>fox")
    assert t.eod in ids
    a2 = _args(tokenizer_type="SentencePieceTokenizer", vocab_file=spm_model, new_tokens=False)
    t2 = build_tokenizer(a2)
    assert t2.vocab_size == n and t2.cls is None


def test_gpt2_bpe_roundtrip(tmp_path):
    pytest.importorskip("transformers")
    # tiny byte-level BPE: bytes of "hello world" + one merge
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("\xa1"), ord("\xac") + 1)) + \
        list(range(ord("\xae"), ord("\xff") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):  # GPT-2's reversible byte -> unicode map
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    b2u = dict(zip(bs, map(chr, cs)))
    chars = sorted({b2u[b] for b in "hello world!".encode()})
    vocab = {c: i for i, c in enumerate(chars)}
    vocab["he"] = len(vocab)
    vocab["<|endoftext|>"] = len(vocab)
    (tmp_path / "vocab.json").write_text(json.dumps(vocab))
    (tmp_path / "merges.txt").write_text("#version: 0.2\nh e\n")
    t = build_tokenizer(_args(tokenizer_type="GPT2BPETokenizer",
                              vocab_file=str(tmp_path / "vocab.json"),
                              merge_file=str(tmp_path / "merges.txt")))
    ids = t.tokenize("hello world!")
    assert ids[0] == vocab["he"] and t.detokenize(ids) == "hello world!"
    assert t.eod == vocab["<|endoftext|>"] and t.vocab_size == len(vocab)


def test_bert_wordpiece(tmp_path):
    pytest.importorskip("transformers")
    toks = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]", "hello", "world", "##s"]
    (tmp_path / "vocab.txt").write_text("\n".join(toks) + "\n")
    t = build_tokenizer(_args(tokenizer_type="BertWordPieceLowerCase",
                              vocab_file=str(tmp_path / "vocab.txt"), vocab_extra_ids=2))
    assert (t.cls, t.sep, t.pad, t.mask) == (2, 3, 0, 4)
    ids = t.tokenize("Hello worlds")
    assert ids == [5, 6, 7]
    assert t.decode_token_ids(ids) == "hello worlds"
    assert len(t.additional_special_tokens_ids) == 2

"""jsonl corpus -> indexed ``.bin/.idx`` (reference ``tools/preprocess_data.py``).

Same CLI as the reference (``--input --json_keys --split_sentences
--keep_newlines --tokenizer_type --vocab_file --merge_file --append_eod --lang
--output_prefix --dataset_impl --workers --chunk_size --log_interval
--vocab_extra_ids --vocab_extra_ids_list --no_new_tokens``) and the same output
naming ``<output_prefix>_<key>_{document,sentence}.{bin,idx}``.

Differences by design:

* tokenisation runs in a process pool over line chunks and each worker returns
  one flat int32 array per document (not a list of Python lists), so the
  parent only memcpys into the builder;
* NLTK is not part of this image: ``--split_sentences`` uses NLTK's punkt when
  importable and otherwise a regex splitter on sentence-final punctuation
  (``--keep_newlines`` keeps the newline attached to the sentence).
"""
import argparse
import json
import multiprocessing
import os
import re
import sys
import time

import numpy as np

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), os.path.pardir)))

from epfl_megatron_amd.data import indexed_dataset  # noqa: E402
from epfl_megatron_amd.tokenizer import build_tokenizer  # noqa: E402

_SENT_END = re.compile(r"(?<=[.!?])(\s+)")


class RegexSentenceSplitter:
    def __init__(self, keep_newlines=False):
        self.keep_newlines = keep_newlines

    def tokenize(self, text):
        parts = _SENT_END.split(text)
        out = []
        for i in range(0, len(parts), 2):
            sent = parts[i]
            if self.keep_newlines and i + 1 < len(parts) and "\n" in parts[i + 1]:
                sent = sent + parts[i + 1][parts[i + 1].index("\n"):]
            if sent.strip():
                out.append(sent)
        return out


class IdentitySplitter:
    def tokenize(self, *text):
        return text


def _make_splitter(args):
    if not args.split_sentences:
        return IdentitySplitter()
    try:
        import nltk
        splitter = nltk.load(f"tokenizers/punkt/{args.lang}.pickle")
        if args.keep_newlines:
            class _Vars(nltk.tokenize.punkt.PunktLanguageVars):
                _period_context_fmt = r"""
                    \S*%(SentEndChars)s\s*(?=(?P<after_tok>%(NonWord)s|(?P<next_tok>\S+)))"""
            return nltk.tokenize.punkt.PunktSentenceTokenizer(train_text=splitter._params,
                                                              lang_vars=_Vars())
        return splitter
    except Exception:
        return RegexSentenceSplitter(args.keep_newlines)


class Encoder:
    def __init__(self, args):
        self.args = args

    def initializer(self):
        Encoder.tokenizer = build_tokenizer(self.args)
        Encoder.splitter = _make_splitter(self.args)

    def encode(self, json_line):
        """-> ({key: (flat int32 tokens, per-sentence sizes)}, bytes read)."""
        data = json.loads(json_line)
        out = {}
        for key in self.args.json_keys:
            sents = [Encoder.tokenizer.tokenize(s) for s in Encoder.splitter.tokenize(data[key])]
            sents = [list(s) for s in sents if len(s) > 0]
            if sents and self.args.append_eod:
                sents[-1].append(Encoder.tokenizer.eod)
            sizes = [len(s) for s in sents]
            flat = np.fromiter((t for s in sents for t in s), dtype=np.int64,
                               count=sum(sizes))
            out[key] = (flat, sizes)
        return out, len(json_line)


def get_args(argv=None):
    p = argparse.ArgumentParser()
    g = p.add_argument_group(title="input data")
    g.add_argument("--input", type=str, required=True, help="Path to input JSON")
    g.add_argument("--json_keys", nargs="+", default=["text"])
    g.add_argument("--split_sentences", action="store_true")
    g.add_argument("--keep_newlines", action="store_true")
    g = p.add_argument_group(title="tokenizer")
    g.add_argument("--tokenizer_type", type=str, required=True,
                   choices=["BertWordPieceLowerCase", "BertWordPieceCase", "GPT2BPETokenizer",
                            "SentencePieceTokenizer", "FalconTokenizer", "NullTokenizer"])
    g.add_argument("--vocab_file", type=str, default=None)
    g.add_argument("--merge_file", type=str, default=None)
    g.add_argument("--tokenizer_model", type=str, default=None)
    g.add_argument("--append_eod", action="store_true")
    g.add_argument("--lang", type=str, default="english")
    g = p.add_argument_group(title="output data")
    g.add_argument("--output_prefix", type=str, required=True)
    g.add_argument("--dataset_impl", type=str, default="mmap", choices=["lazy", "cached", "mmap"])
    g = p.add_argument_group(title="runtime")
    g.add_argument("--workers", type=int, required=True)
    g.add_argument("--chunk_size", type=int, required=True)
    g.add_argument("--log_interval", type=int, default=100)
    g.add_argument("--vocab_extra_ids", type=int, default=0)
    g.add_argument("--vocab_extra_ids_list", type=str, default=None)
    g.add_argument("--no_new_tokens", action="store_false", dest="new_tokens")
    g.add_argument("--synthetic_vocab_size", type=int, default=32000,
                   help="vocab of the NullTokenizer (whitespace-separated integer ids)")
    args = p.parse_args(argv)
    args.keep_empty = False
    if args.tokenizer_type.lower().startswith("bert") and not args.split_sentences:
        print("Bert tokenizer detected, are you sure you don't want to split sentences?")
    args.rank = 0
    args.make_vocab_size_divisible_by = 128
    args.tensor_model_parallel_size = 1
    return args


def main(argv=None):
    args = get_args(argv)
    t_start = time.time()
    print("Opening", args.input)
    encoder = Encoder(args)
    tokenizer = build_tokenizer(args)
    level = "sentence" if args.split_sentences else "document"
    print(f"Vocab size: {tokenizer.vocab_size}")
    print(f"Output prefix: {args.output_prefix}")
    builders, idx_files = {}, {}
    for key in args.json_keys:
        stem = f"{args.output_prefix}_{key}_{level}"
        idx_files[key] = stem + ".idx"
        builders[key] = indexed_dataset.make_builder(stem + ".bin", impl=args.dataset_impl,
                                                     vocab_size=tokenizer.vocab_size)
    with open(args.input, "r", encoding="utf-8") as fin:
        if args.workers > 1:
            pool = multiprocessing.get_context("fork").Pool(args.workers,
                                                            initializer=encoder.initializer)
            docs = pool.imap(encoder.encode, fin, args.chunk_size)
        else:
            pool = None
            encoder.initializer()
            docs = map(encoder.encode, fin)
        print("Time to startup:", time.time() - t_start)
        t0 = time.time()
        nbytes = 0
        for i, (doc, nb) in enumerate(docs, start=1):
            nbytes += nb
            for key, (flat, sizes) in doc.items():
                if not sizes:
                    continue
                b = builders[key]
                if isinstance(b, indexed_dataset.MMapIndexedDatasetBuilder):
                    b.add_doc(flat, sizes)
                else:
                    off = 0
                    for s in sizes:
                        b.add_item(flat[off:off + s])
                        off += s
                    b.end_document()
            if i % args.log_interval == 0:
                el = time.time() - t0
                print(f"Processed {i} documents ({i / el:.1f} docs/s, "
                      f"{nbytes / el / 1024 / 1024:.2f} MB/s).", file=sys.stderr)
        if pool is not None:
            pool.close()
            pool.join()
    print("Done! Now finalizing.")
    for key in args.json_keys:
        builders[key].finalize(idx_files[key])


if __name__ == "__main__":
    main()

"""Byte-level BPE (GPT-2 vocab.json + merges.txt), self-contained.

Role of the reference's vendored ``megatron/tokenizer/gpt2_tokenization.py``:
no network, no dependency on a particular ``transformers`` version (whose
GPT-2 tokenizer API changed).  Same algorithm and outputs as GPT-2's
encoder: the reversible byte -> unicode map, the GPT-2 pre-tokenisation
regex, and greedy lowest-rank pair merging, with a per-word cache.
"""
import json
from functools import lru_cache

import regex as re

_PAT = re.compile(r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+""")


@lru_cache()
def bytes_to_unicode():
    """Map every byte to a printable unicode character (GPT-2's table)."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("\xa1"), ord("\xac") + 1)) + \
        list(range(ord("\xae"), ord("\xff") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, map(chr, cs)))


def _pairs(word):
    return {(word[i], word[i + 1]) for i in range(len(word) - 1)}


class GPT2BPE:

    def __init__(self, vocab_file, merges_file, errors="replace"):
        with open(vocab_file, encoding="utf-8") as f:
            self.encoder = json.load(f)
        self.decoder = {v: k for k, v in self.encoder.items()}
        with open(merges_file, encoding="utf-8") as f:
            lines = f.read().split("\n")
        merges = [tuple(ln.split()) for ln in lines
                  if ln and not ln.startswith("#version") and len(ln.split()) == 2]
        self.bpe_ranks = {m: i for i, m in enumerate(merges)}
        self.byte_encoder = bytes_to_unicode()
        self.byte_decoder = {v: k for k, v in self.byte_encoder.items()}
        self.errors = errors
        self.cache = {}

    def bpe(self, token):
        if token in self.cache:
            return self.cache[token]
        word = tuple(token)
        pairs = _pairs(word)
        if not pairs:
            return [token]
        while True:
            bigram = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if bigram not in self.bpe_ranks:
                break
            first, second = bigram
            new, i = [], 0
            while i < len(word):
                try:
                    j = word.index(first, i)
                except ValueError:
                    new.extend(word[i:])
                    break
                new.extend(word[i:j])
                i = j
                if i < len(word) - 1 and word[i] == first and word[i + 1] == second:
                    new.append(first + second)
                    i += 2
                else:
                    new.append(word[i])
                    i += 1
            word = tuple(new)
            if len(word) == 1:
                break
            pairs = _pairs(word)
        out = list(word)
        if len(self.cache) < 1 << 20:
            self.cache[token] = out
        return out

    def encode(self, text):
        ids = []
        for tok in _PAT.findall(text):
            t = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
            ids.extend(self.encoder[p] for p in self.bpe(t))
        return ids

    def decode(self, ids):
        text = "".join(self.decoder[int(i)] for i in ids)
        return bytearray(self.byte_decoder[c] for c in text).decode("utf-8", errors=self.errors)

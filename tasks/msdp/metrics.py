"""Dialogue metrics for MSDP (reference ``tasks/msdp/metrics.py``).

Token-level precision / recall / F1 after SQuAD-style normalisation (lower
case, punctuation -> space, articles dropped, whitespace collapsed).  Pairs
whose gold side is empty are skipped; an empty guess scores 0.  Also holds a
dependency-free word tokenizer used wherever the reference calls
``nltk.word_tokenize`` (nltk is not part of this image).
"""
import re
from collections import Counter

_ARTICLES = re.compile(r"\b(a|an|the)\b")
_PUNCT = re.compile(r"[!\"#$%&()*+,\-./:;<=>?@\[\]\\^`{|}~_']")

# Penn-Treebank-style splitting: clitics, punctuation and quotes become tokens.
_CLITICS = re.compile(r"(?i)(\w)(n't|'s|'re|'ve|'ll|'d|'m)\b")
_TOKEN = re.compile(r"n't|'(?:s|re|ve|ll|d|m)\b|\w+(?:[-.]\w+)*|\.\.\.|[^\w\s]", re.IGNORECASE)


def word_tokenize(text):
    """Split ``text`` into word / punctuation tokens (``"don't stop."`` ->
    ``["do", "n't", "stop", "."]``)."""
    text = _CLITICS.sub(r"\1 \2", text)
    return _TOKEN.findall(text)


def normalize_answer(s):
    s = _PUNCT.sub(" ", s.lower())
    s = _ARTICLES.sub(" ", s)
    return " ".join(s.split())


def _prf(pred, gold):
    same = sum((Counter(gold) & Counter(pred)).values())
    if same == 0:
        return 0.0, 0.0, 0.0
    p, r = same / len(pred), same / len(gold)
    return p, r, 2 * p * r / (p + r)


class F1Metric:
    @staticmethod
    def compute_each_pair(guess, answer):
        if answer == "":
            return None, None, None
        if guess == "":
            return 0.0, 0.0, 0.0
        return _prf(normalize_answer(guess).split(), normalize_answer(answer).split())

    @staticmethod
    def compute_all_pairs(guesses, answers):
        assert len(guesses) == len(answers), "lengths of guesses and answers differ"
        scores = [F1Metric.compute_each_pair(g, a) for g, a in zip(guesses, answers)]
        scores = [s for s in scores if s[0] is not None]
        if not scores:
            return 0.0, 0.0, 0.0
        n = len(scores)
        return tuple(sum(s[i] for s in scores) / n for i in range(3))

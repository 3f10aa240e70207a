"""Retrieval answer matching (reference ``tasks/orqa/unsupervised/qa_utils.py``,
the DPR validation protocol).

``calculate_matches`` checks, for each question, which of its retrieved
passages contain an answer (token-sequence match after NFD normalisation and
lower-casing, or a regex search) and accumulates ``top_k_hits[k-1]`` = number
of questions answered within the first k passages.
"""
import collections
import string
import unicodedata
from functools import partial
from multiprocessing import Pool

import regex

from .tokenizers import SimpleTokenizer

QAMatchStats = collections.namedtuple("QAMatchStats", ["top_k_hits", "questions_doc_hits"])

_DOCS = None


def _normalize(text):
    return unicodedata.normalize("NFD", text)


def regex_match(text, pattern):
    try:
        pat = regex.compile(pattern, flags=regex.IGNORECASE + regex.UNICODE + regex.MULTILINE)
    except Exception:
        return False
    return pat.search(text) is not None


def has_answer(answers, text, tokenizer, match_type):
    text = _normalize(text)
    if match_type == "string":
        words = tokenizer.tokenize(text).words(uncased=True)
        for ans in answers:
            a = tokenizer.tokenize(_normalize(ans)).words(uncased=True)
            n = len(a)
            if any(words[i:i + n] == a for i in range(len(words) - n + 1)):
                return True
    elif match_type == "regex":
        return any(regex_match(text, _normalize(ans)) for ans in answers)
    return False


def check_answer(question_answers_docs, tokenizer, match_type, docs=None):
    answers, (doc_ids, _scores) = question_answers_docs
    docs = docs if docs is not None else _DOCS
    hits = []
    for d in doc_ids:
        doc = docs.get(d) if hasattr(docs, "get") else docs[d]
        hits.append(doc is not None and doc[0] is not None and
                    has_answer(answers, doc[0], tokenizer, match_type))
    return hits


def _init_worker(docs):
    global _DOCS
    _DOCS = docs


def calculate_matches(all_docs, answers, closest_docs, workers_num, match_type):
    tok = SimpleTokenizer()
    pairs = list(zip(answers, closest_docs))
    if workers_num and workers_num > 1:
        with Pool(workers_num, initializer=_init_worker, initargs=(all_docs,)) as pool:
            scores = pool.map(partial(check_answer, tokenizer=tok, match_type=match_type), pairs)
    else:
        scores = [check_answer(p, tok, match_type, docs=all_docs) for p in pairs]
    n_docs = len(closest_docs[0][0]) if closest_docs else 0
    top_k_hits = [0] * n_docs
    for hits in scores:
        best = next((i for i, h in enumerate(hits) if h), None)
        if best is not None:
            for i in range(best, n_docs):
                top_k_hits[i] += 1
    return QAMatchStats(top_k_hits, scores)


def _normalize_answer(s):
    s = "".join(ch for ch in s.lower() if ch not in set(string.punctuation))
    s = regex.sub(r"\b(a|an|the)\b", " ", s)
    return " ".join(s.split())


def exact_match_score(prediction, ground_truth):
    return _normalize_answer(prediction) == _normalize_answer(ground_truth)

"""Remove downstream-task n-gram overlaps from a training corpus (reference
``tools/openwebtext/filter_ngrams.py``).

    python filter_ngrams.py --tasks lambada --lambada_path lambada_test.jsonl \
        --task_files extra_eval.txt --dedup_dataset train.json text --output clean.json

Task n-grams are ``--max_ngram_size`` lower-cased ``\\w+`` words (a task text
shorter than that but with at least ``--min_ngram_size`` words contributes
itself whole).  When a training document contains one, it is split there: the
n-gram plus ``--remove_char_each_side`` characters on each side are cut,
extended outwards to the nearest sentence end (reference ``split_text``
:29-49), and both halves are checked again.  Pieces shorter than
``--filter_text_char_len`` characters are dropped; a document split more than
``--splits_count`` times is dropped entirely.

Task sources: the reference pulls SQuAD/RACE/... through the ``datasets``
hub, which is unreachable here; instead any local eval file can be given with
``--task_files`` (jsonl with a ``text`` field, or plain text, one example per
line).  The frequency-threshold shrinking of frequent n-grams
(``--key_threshold``) is not reproduced (parity unpinned).
"""
import argparse
import json
import re

_WORD = re.compile(r"\w+")
PUNCT = ".!?"


def get_words(text):
    ws, pos = [], []
    for m in _WORD.finditer(text.lower()):
        ws.append(m.group(0))
        pos.append(m.start())
    return ws, pos


def task_ngrams(texts, max_n=13, min_n=8):
    grams = set()
    for t in texts:
        w, _ = get_words(t)
        if len(w) >= max_n:
            grams.update(" ".join(w[i:i + max_n]) for i in range(len(w) - max_n + 1))
        elif len(w) >= min_n:
            grams.add(" ".join(w))
    return grams


def split_text(text, start, end, remove_each_side):
    """Text before ``start - remove`` (cut back to a sentence end) and after
    ``end + remove`` (cut forward past the next sentence end)."""
    pos = start - remove_each_side
    while pos > 0 and text[pos] not in PUNCT:
        pos -= 1
    first = text[:pos + 1] if pos > 0 else ""
    pos = end + remove_each_side
    while pos < len(text) and text[pos] not in PUNCT:
        pos += 1
    second = text[pos + 1:] if pos + 1 < len(text) else ""
    return first, second


def _first_match(text, grams, sizes):
    w, pos = get_words(text)
    for i in range(len(w)):
        for n in sizes:
            if i + n <= len(w) and " ".join(w[i:i + n]) in grams:
                last = i + n - 1
                return pos[i], pos[last] + len(w[last])
    return None


def clean_document(text, grams, sizes, remove_each_side=200, min_chars=200, max_splits=10):
    """-> (kept pieces, number of splits); ``[]`` when the document is dropped."""
    pieces, todo, splits = [], [text], 0
    while todo:
        t = todo.pop(0)
        m = _first_match(t, grams, sizes)
        if m is None:
            if len(t) >= min_chars:
                pieces.append(t)
            continue
        splits += 1
        if splits > max_splits:
            return [], splits
        a, b = split_text(t, m[0], m[1], remove_each_side)
        if len(a) >= min_chars:
            pieces.append(a)
        if b:
            todo.append(b)
    return pieces, splits


def _read_task_file(path):
    out = []
    with open(path, encoding="utf-8") as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            try:
                d = json.loads(line)
                out.append(d["text"] if isinstance(d, dict) else str(d))
            except ValueError:
                out.append(line)
    return out


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--tasks", nargs="*", default=[])
    p.add_argument("--lambada_path", type=str, default=None)
    p.add_argument("--task_files", nargs="*", default=[])
    p.add_argument("--dedup_dataset", nargs=2, required=True, metavar=("FILE", "KEY"))
    p.add_argument("--output", type=str, required=True)
    p.add_argument("--max_ngram_size", type=int, default=13)
    p.add_argument("--min_ngram_size", type=int, default=8)
    p.add_argument("--filter_text_char_len", type=int, default=200)
    p.add_argument("--splits_count", type=int, default=10)
    p.add_argument("--remove_char_each_side", type=int, default=200)
    p.add_argument("--key_threshold", type=int, default=10, help="accepted; unused")
    a = p.parse_args(argv)
    texts = []
    if "lambada" in a.tasks:
        assert a.lambada_path, "--lambada_path is required for the lambada task"
        texts += _read_task_file(a.lambada_path)
    for f in a.task_files:
        texts += _read_task_file(f)
    grams = task_ngrams(texts, a.max_ngram_size, a.min_ngram_size)
    sizes = sorted({len(g.split()) for g in grams}, reverse=True)
    path, key = a.dedup_dataset
    st = dict(docs=0, clean=0, split=0, dropped=0, pieces=0)
    with open(path, encoding="utf-8") as fin, open(a.output, "w", encoding="utf-8") as fout:
        for line in fin:
            doc = json.loads(line)
            st["docs"] += 1
            pieces, n = clean_document(doc[key], grams, sizes, a.remove_char_each_side,
                                       a.filter_text_char_len, a.splits_count)
            st["clean" if n == 0 else "split"] += 1
            st["dropped"] += not pieces
            for i, piece in enumerate(pieces):
                out = dict(doc)
                out[key] = piece
                if n:
                    out["split_id"] = i
                fout.write(json.dumps(out, ensure_ascii=False) + "\n")
                st["pieces"] += 1
    print(f"{len(grams)} task n-grams | {st}", flush=True)
    return st


if __name__ == "__main__":
    main()

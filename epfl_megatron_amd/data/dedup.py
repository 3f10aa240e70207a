"""Near-duplicate document detection (backs ``tools/openwebtext``).

Reference: ``tools/openwebtext/find_duplicates.py`` (MinHash + LSH buckets via
the external ``lsh`` package, Jaccard over character 5-gram shingles,
``url_pairs_to_remove`` :63-104 with the ``--heuristic_iter`` shortcut) and
``group_duplicate_url.py`` (union of pairs above a threshold into groups).

Fingerprints are saved as ``.npz`` (ids, texts, signatures) instead of
pickles, so loading a fingerprint file never executes code.
"""
import json

import numpy as np

try:
    from . import _dedup
except ImportError:  # fresh checkout: compile the CPU module in-tree once
    from ..build import build_dedup
    build_dedup()
    from . import _dedup

JACCARD_MODES = {"union": 0, "min": 1, "max": 2}


class LSHIndex:
    """MinHash signatures of documents, bucketed by LSH band keys."""

    def __init__(self, num_seeds=100, num_bands=10, seed=1234, char_ngram=5, threads=8):
        assert num_seeds % num_bands == 0, "num_seeds must be divisible by num_bands"
        self.seeds = np.random.RandomState(seed).randint(0, 10 ** 6, size=num_seeds).astype(np.int64)
        self.num_bands, self.char_ngram, self.threads = num_bands, char_ngram, threads
        self.ids, self.texts = [], []
        self.signatures = np.zeros((0, num_seeds), dtype=np.uint32)

    def add(self, ids, texts):
        sig = _dedup.minhash(list(texts), self.seeds, self.char_ngram, self.threads)
        self.ids.extend(ids)
        self.texts.extend(texts)
        self.signatures = np.concatenate([self.signatures, sig])

    def buckets(self):
        """Per band: list of index groups (size > 1) sharing that band's key."""
        keys = _dedup.band_keys(self.signatures, self.num_bands)
        out = []
        for b in range(self.num_bands):
            order = np.argsort(keys[:, b], kind="stable")
            k = keys[order, b]
            cuts = np.flatnonzero(np.diff(k)) + 1
            out.append([g.tolist() for g in np.split(order, cuts) if len(g) > 1])
        return out

    def save(self, path):
        np.savez(path, ids=np.array(self.ids, dtype=object).astype(str),
                 texts=np.array(self.texts, dtype=object).astype(str),
                 signatures=self.signatures, seeds=self.seeds,
                 meta=np.array([self.num_bands, self.char_ngram]))

    def merge_file(self, path):
        z = np.load(path if path.endswith(".npz") else path + ".npz", allow_pickle=False)
        assert np.array_equal(z["seeds"], self.seeds), "fingerprints use different seeds"
        self.ids.extend(z["ids"].tolist())
        self.texts.extend(z["texts"].tolist())
        self.signatures = np.concatenate([self.signatures, z["signatures"]])


def jaccard(a, b, mode="union", char_ngram=5):
    return _dedup.jaccard(a, b, char_ngram, JACCARD_MODES[mode])


def pairs_to_remove(bucket, texts, ids, rng, mode="union", heuristic_iter=1, threshold=0.5):
    """Greedy pass over one bucket (reference ``url_pairs_to_remove``): pick a
    random main document, mark every other with Jaccard > ``threshold`` as its
    duplicate, drop them and the main from the bucket, repeat
    (``heuristic_iter`` times, -1 = until the bucket is empty)."""
    bucket = list(bucket)
    found, it = [], 0
    while len(bucket) > 1 and it != heuristic_iter:
        main = bucket[rng.randint(0, len(bucket))]
        dups = []
        for other in bucket:
            if other != main:
                s = jaccard(texts[main], texts[other], mode)
                if s > threshold:
                    dups.append((other, s))
        drop = {o for o, _ in dups} | {main}
        bucket = [x for x in bucket if x not in drop]
        if dups:
            found.append({ids[main]: [{ids[o]: s} for o, s in dups]})
        it += 1
    return found


def find_duplicates(index, mode="union", heuristic_iter=1, seed=1234):
    rng = np.random.RandomState(seed)
    out = []
    for band in index.buckets():
        for bucket in band:
            out.extend(pairs_to_remove(bucket, index.texts, index.ids, rng, mode, heuristic_iter))
    return out


def group_duplicates(pair_lines, threshold=0.7):
    """Union pairs with similarity >= ``threshold`` into groups of urls
    (reference ``group_duplicate_url.py``); returns a list of sets, size > 1."""
    parent = {}

    def find(x):
        parent.setdefault(x, x)
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for entry in pair_lines:
        if isinstance(entry, str):
            entry = json.loads(entry)
        for main, others in entry.items():
            find(main)
            for o in others:
                for url, sim in o.items():
                    if sim >= threshold:
                        parent[find(url)] = find(main)
    groups = {}
    for x in list(parent):
        groups.setdefault(find(x), set()).add(x)
    return [g for g in groups.values() if len(g) > 1]

"""Exercise every entry point of the native CPU helpers and save the results.

Run twice by ``tests/test_sanitizers.py``: once inside the sanitizer harness
(``csrc/sanitize_main.cpp``, where ``_helpers``/``_dedup`` are embedded
modules built with ASan+UBSan or TSan) and once with the normal in-tree
extensions; the two result files must match and the sanitized run must not
report.  Inputs include the edge cases the index builders must survive: empty
and one-token documents, a sample ending exactly on a document boundary,
single-sentence documents, weights with a zero entry, empty texts.

    sanitize_driver.py OUT.npz [embedded|package]
"""
import sys

import numpy as np


def _modules(mode):
    if mode == "embedded":
        import _dedup  # noqa: F401  (embedded in the harness executable)
        import _helpers
        return _helpers, _dedup
    from epfl_megatron_amd.data import _dedup, _helpers
    return _helpers, _dedup


def run(helpers, dedup):
    out = {}
    rng = np.random.default_rng(1234)
    sizes = rng.integers(0, 40, size=200).astype(np.int32)
    sizes[[0, 7, 8]] = [0, 1, 0]
    doc_idx = np.concatenate([rng.permutation(200) for _ in range(3)]).astype(np.int32)
    tokens_per_epoch = int(sizes.sum())
    for seq in (16, 31, tokens_per_epoch - 1):
        out[f"sample_idx_{seq}"] = helpers.sample_index(sizes, doc_idx, seq, 3, tokens_per_epoch)

    for w in ([0.5, 0.3, 0.2], [0.0, 1.0], [1.0]):
        which, within = helpers.blend_indices(np.array(w, dtype=np.float64), 997, False)
        out[f"blend_{len(w)}_{w[0]}"] = np.stack([which.astype(np.int64), within.astype(np.int64)])

    pointers = np.concatenate([[0], np.cumsum(sizes[:-1].astype(np.int64))]) * 4
    toks = rng.integers(0, 50000, size=int(sizes.sum())).astype(np.int32)
    sidx = out["sample_idx_16"]
    samples = np.arange(len(sidx) - 1, dtype=np.int64)
    out["stitch"] = helpers.stitch_samples(toks, pointers, sizes, doc_idx, sidx, samples, 16)

    nsent = rng.integers(1, 6, size=60)
    docs = np.concatenate([[0], np.cumsum(nsent)]).astype(np.int64)
    ssizes = rng.integers(1, 30, size=int(docs[-1])).astype(np.int32)
    ssizes[3] = 500  # a sentence longer than any sample
    for prob in (0.0, 0.3):
        out[f"pairs_{prob}"] = np.asarray(helpers.sentence_pair_mapping(
            docs, ssizes, 2, 10000, 48, prob, 7, False, 2)).astype(np.int64)
    titles = rng.integers(1, 8, size=60).astype(np.int32)
    for one in (False, True):
        out[f"blocks_{one}"] = np.asarray(helpers.block_mapping(
            docs, ssizes, titles, 2, 10000, 64, 7, False, one)).astype(np.int64)

    texts = ["", "abc", "the quick brown fox jumps over the lazy dog" * 3,
             "the quick brown fox jumped over the lazy dogs" * 3, "éèê unicode ✓ text " * 5]
    texts += ["".join(chr(97 + int(c)) for c in rng.integers(0, 26, size=300)) for _ in range(40)]
    seeds = np.arange(1, 65, dtype=np.int64)
    sig = dedup.minhash(texts, seeds, 5, 4)
    out["minhash"] = sig.astype(np.int64)
    out["bands"] = dedup.band_keys(sig, 8).view(np.int64)
    out["jaccard"] = np.array([dedup.jaccard(texts[i], texts[j], 5, m)
                               for i in range(5) for j in range(5) for m in range(3)])
    return out


def main():
    path, mode = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "package")
    res = run(*_modules(mode))
    np.savez(path, **res)
    print(f"sanitize_driver: {len(res)} results -> {path}")


if __name__ == "__main__":
    main()

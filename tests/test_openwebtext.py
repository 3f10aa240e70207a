"""Corpus-cleaning tools (tools/openwebtext) and the native MinHash/LSH module.

The reference's tools have no tests and depend on packages absent here
(``lsh``, ``ftfy``, ``langdetect``, ``tldextract``); expectations below follow
the reference's rules on synthetic documents (parity unpinned for the exact
hash values, which differ from the ``lsh`` package's murmur3 by design).
"""
import json
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OWT = os.path.join(ROOT, "tools", "openwebtext")
sys.path.insert(0, ROOT)
sys.path.insert(0, OWT)

from epfl_megatron_amd.data import dedup  # noqa: E402


def _shingles(t, n=5):
    return {t[h:h + n] for h in range(0, len(t) - n)}


def _doc(rng, n=400):
    words = "alpha beta gamma delta epsilon zeta eta theta iota kappa lambda mu nu xi".split()
    return " ".join(rng.choice(words) + str(rng.randint(0, 50)) for _ in range(n // 6))


def test_jaccard_matches_python_sets():
    rng = random.Random(0)
    a = _doc(rng)
    b = a[:300] + _doc(rng)[:100] + " ünïcödé ✓"
    sa, sb = _shingles(a), _shingles(b)
    ref = {"union": len(sa & sb) / len(sa | sb), "min": len(sa & sb) / min(len(sa), len(sb)),
           "max": len(sa & sb) / max(len(sa), len(sb))}
    for mode, v in ref.items():
        assert dedup.jaccard(a, b, mode) == pytest.approx(v, abs=1e-12)
    assert dedup.jaccard("abc", a) == 0.0


def test_minhash_estimates_jaccard():
    rng = random.Random(1)
    a = _doc(rng, 3000)
    b = a[:2000] + _doc(rng, 1000)
    idx = dedup.LSHIndex(num_seeds=256, num_bands=16)
    idx.add(["a", "b"], [a, b])
    est = float(np.mean(idx.signatures[0] == idx.signatures[1]))
    assert est == pytest.approx(dedup.jaccard(a, b), abs=0.1)
    # deterministic across thread counts
    idx2 = dedup.LSHIndex(num_seeds=256, num_bands=16, threads=1)
    idx2.add(["a", "b"], [a, b])
    assert np.array_equal(idx.signatures, idx2.signatures)


def _corpus(tmp_path):
    rng = random.Random(2)
    base = [_doc(rng, 1200) for _ in range(6)]
    docs = [{"url": f"u{i}", "text": t} for i, t in enumerate(base)]
    docs.append({"url": "dup0", "text": base[0][:-10] + " tail."})  # near-duplicate of u0
    docs.append({"url": "dup3", "text": base[3]})  # exact duplicate of u3
    path = tmp_path / "docs.json"
    path.write_text("".join(json.dumps(d) + "\n" for d in docs))
    return path, docs


def test_dedup_pipeline(tmp_path):
    import find_duplicates
    import group_duplicate_url
    import remove_group_duplicates
    path, docs = _corpus(tmp_path)
    pairs, fp = tmp_path / "pairs.json", tmp_path / "fp.npz"
    find_duplicates.main(["--inputs", str(path), "url", "--output", str(pairs),
                          "--save_fingerprints", str(fp), "--heuristic_iter", "-1"])
    found = [json.loads(x) for x in pairs.read_text().splitlines()]
    flat = {frozenset([m, list(o)[0]]) for e in found for m, os_ in e.items() for o in os_}
    assert flat == {frozenset(["u0", "dup0"]), frozenset(["u3", "dup3"])}
    # reload fingerprints (pickle-free) -> same result
    pairs2 = tmp_path / "pairs2.json"
    find_duplicates.main(["--load_fingerprints", str(fp), "--output", str(pairs2),
                          "--heuristic_iter", "-1"])
    found2 = [json.loads(x) for x in pairs2.read_text().splitlines()]
    assert {frozenset([m, list(o)[0]]) for e in found2 for m, os_ in e.items() for o in os_} == flat
    groups = tmp_path / "groups.json"
    group_duplicate_url.main([str(pairs), str(groups)])
    g = [sorted(list(json.loads(x).values())[0]) for x in groups.read_text().splitlines()]
    assert sorted(g) == [["dup0", "u0"], ["dup3", "u3"]]
    out = tmp_path / "dedup.json"
    written, removed = remove_group_duplicates.main([str(groups), str(path), str(out)])
    assert (written, removed) == (6, 2)
    kept = {json.loads(x)["url"] for x in out.read_text().splitlines()}
    assert kept == {"u1", "u2", "u4", "u5", "dup0", "dup3"}  # sorted group -> first kept


def test_group_duplicates_union_find():
    lines = [{"a": [{"b": 0.9}, {"c": 0.5}]}, {"c": [{"d": 0.8}]}, {"b": [{"e": 0.71}]}]
    groups = dedup.group_duplicates(lines, 0.7)
    assert sorted(sorted(g) for g in groups) == [["a", "b", "e"], ["c", "d"]]


def test_filter_ngrams(tmp_path):
    import filter_ngrams as fn
    task = "the quick brown fox jumps over the lazy dog while the cat sleeps on the mat"
    grams = fn.task_ngrams([task], 13, 8)
    sizes = sorted({len(g.split()) for g in grams}, reverse=True)
    pre = "First sentence here. " * 20
    post = " Later text continues. " * 20
    doc = pre + "Yes, The quick brown fox jumps over the lazy dog while the cat sleeps on." + post
    pieces, n = fn.clean_document(doc, grams, sizes, remove_each_side=30, min_chars=50)
    assert n == 1 and len(pieces) == 2
    assert "fox" not in pieces[0] + pieces[1]
    assert pieces[0].endswith(".") and doc.startswith(pieces[0])
    assert doc.endswith(pieces[1])
    clean, n0 = fn.clean_document(pre, grams, sizes, min_chars=50)
    assert n0 == 0 and clean == [pre]
    # too many splits -> dropped
    many = (pre + task + ". ") * 4
    assert fn.clean_document(many, grams, sizes, 10, 10, max_splits=2) == ([], 3)
    # CLI end-to-end
    data, lam, out = tmp_path / "d.json", tmp_path / "l.jsonl", tmp_path / "o.json"
    data.write_text(json.dumps({"text": doc, "id": 1}) + "\n" + json.dumps({"text": pre, "id": 2}) + "\n")
    lam.write_text(json.dumps({"text": task}) + "\n")
    st = fn.main(["--tasks", "lambada", "--lambada_path", str(lam), "--dedup_dataset", str(data),
                  "text", "--output", str(out), "--remove_char_each_side", "30",
                  "--filter_text_char_len", "50"])
    assert st == dict(docs=2, clean=1, split=1, dropped=0, pieces=3)


def test_cleanup_and_url_tools(tmp_path):
    import add_id
    import blacklist_urls as bl
    import cleanup_fix_dataset as cf
    import textclean
    assert cf.process_doc("short", ["remove_512"]) == ("remove_512", "short", True)
    assert cf.process_doc("x" * 600 + "  y\n z", ["general_cleaning"])[1] == "x" * 600 + " y z"
    assert cf.process_doc("go javascript", ["remove_256_javascript"])[2]
    assert textclean.is_english("This is the best thing that has ever been written about it.")
    assert not textclean.is_english("Dies ist ein völlig deutscher Satz über nichts Besonderes.")
    seen = set()
    assert bl.classify("https://www.youtube.com/watch?v=1", seen) == "domain"
    assert bl.classify("https://news.bbc.co.uk/a", seen) == "domain"
    assert bl.classify("https://example.com/a.pdf", seen) == "extension"
    assert bl.classify("http://x", seen) == "short"
    assert bl.classify("https://exa mple.com/a", seen) == "malformed"
    assert bl.classify("https://example.com/story", seen) is None
    seen.add("https://example.com/story")
    assert bl.classify("https://example.com/story", seen) == "duplicate"
    src, dst = tmp_path / "in.json", tmp_path / "out.json"
    src.write_text('{"text": "a"}\n{"text": "b"}\n')
    add_id.main(["--input_file", str(src), "--output_file", str(dst), "--id_prefix", "cc"])
    assert [json.loads(x)["adlr_id"] for x in dst.read_text().splitlines()] == \
        ["cc-0000000001", "cc-0000000002"]

"""Find near-duplicate documents with MinHash + LSH (reference
``tools/openwebtext/find_duplicates.py``).

    python find_duplicates.py --inputs cc.json cc_id news.json news_id \
        --output possible_dups.json [--save_fingerprints fp.npz] [--load_fingerprints a.npz ...]

Fingerprinting and Jaccard run in the native ``_dedup`` module
(``epfl_megatron_amd/csrc/dedup.cpp``, threaded, GIL released).  Output lines:
``{main_id: [{dup_id: jaccard}, ...]}``.  Fingerprint files are ``.npz``.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from epfl_megatron_amd.data.dedup import LSHIndex, find_duplicates  # noqa: E402


def read_docs(path, key):
    ids, texts = [], []
    with open(path, encoding="utf-8") as f:
        for line in f:
            try:
                d = json.loads(line)
                ids.append(d[key])
                texts.append(d["text"])
            except (ValueError, KeyError) as e:
                print("Error:", e)
    return ids, texts


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--inputs", nargs="*", default=None,
                   help="pairs of input file and id key, e.g. cc.json cc_id news.json news_id")
    p.add_argument("--load_fingerprints", nargs="*", default=None)
    p.add_argument("--save_fingerprints", type=str, default=None)
    p.add_argument("--output", type=str, default=None)
    p.add_argument("--jaccard", type=str, default="union", choices=["union", "min", "max"])
    p.add_argument("--heuristic_iter", type=int, default=1, help="-1 for exact")
    p.add_argument("--num_bands", type=int, default=10)
    p.add_argument("--num_seeds", type=int, default=100)
    p.add_argument("--num_threads", type=int, default=min(16, os.cpu_count() or 1))
    p.add_argument("--jaccard_parallel", action="store_true",
                   help="accepted for CLI compatibility (fingerprinting is always threaded)")
    a = p.parse_args(argv)
    t0 = time.time()
    index = LSHIndex(a.num_seeds, a.num_bands, a.seed, threads=a.num_threads)
    for fp in a.load_fingerprints or []:
        print(f"Loading fingerprints from {fp}", flush=True)
        index.merge_file(fp)
    if a.inputs:
        assert len(a.inputs) % 2 == 0, "--inputs takes (file, key) pairs"
        for path, key in zip(a.inputs[::2], a.inputs[1::2]):
            ids, texts = read_docs(path, key)
            index.add(ids, texts)
            print(f" fingerprinted {len(ids)} documents of {path} in {time.time() - t0:.2f} s",
                  flush=True)
    if a.save_fingerprints:
        index.save(a.save_fingerprints)
    if a.output:
        found = find_duplicates(index, a.jaccard, a.heuristic_iter, a.seed)
        with open(a.output, "w", encoding="utf-8") as f:
            for entry in found:
                f.write(json.dumps(entry, ensure_ascii=False) + "\n")
        print(f" {sum(len(v) for e in found for v in e.values())} possible duplicates "
              f"in {time.time() - t0:.2f} s", flush=True)
    print("done :-)")


if __name__ == "__main__":
    main()

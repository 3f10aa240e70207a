"""Group near-duplicate urls (reference ``tools/openwebtext/group_duplicate_url.py``).

    python group_duplicate_url.py possible_dups.json groups.json [threshold=0.7]

Each output line is ``{"<group id>": [kept_url, removed_url, ...]}``; urls are
sorted so the kept one (the first) is deterministic.
"""
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from epfl_megatron_amd.data.dedup import group_duplicates  # noqa: E402


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    threshold = float(argv[2]) if len(argv) > 2 else 0.7
    with open(argv[0], encoding="utf-8") as f:
        groups = group_duplicates((line for line in f if line.strip()), threshold)
    remove = sum(len(g) - 1 for g in groups)
    print(f"{len(groups)} groups: keep {len(groups)}, remove {remove} urls")
    with open(argv[1], "w", encoding="utf-8") as f:
        for i, g in enumerate(groups):
            f.write(json.dumps({str(i): sorted(g)}, ensure_ascii=False) + "\n")


if __name__ == "__main__":
    main()

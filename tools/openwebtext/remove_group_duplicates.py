"""Drop all but the first url of every duplicate group (reference
``tools/openwebtext/remove_group_duplicates.py``).

    python remove_group_duplicates.py groups.json data.json deduped.json
"""
import json
import sys


def main(argv=None):
    url_file, data_file, out_file = (sys.argv[1:] if argv is None else argv)[:3]
    remove = set()
    with open(url_file, encoding="utf-8") as f:
        for line in f:
            for urls in json.loads(line).values():
                remove.update(urls[1:])
    written = removed = removed_chars = 0
    with open(data_file, encoding="utf-8") as fin, open(out_file, "w", encoding="utf-8") as fout:
        for line in fin:
            try:
                d = json.loads(line)
            except ValueError as e:
                print("[SKIPPING]", line, e)
                continue
            if d.get("url") in remove:
                removed += 1
                removed_chars += len(d.get("text", ""))
                continue
            fout.write(json.dumps(d, ensure_ascii=False) + "\n")
            written += 1
    print(f" [PROCESSED] written: {written} | removed: {removed} (char: {removed_chars})")
    return written, removed


if __name__ == "__main__":
    main()

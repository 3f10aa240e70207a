"""Task-selectable document filters / fixes (reference
``tools/openwebtext/cleanup_fix_dataset.py:23-83``).

    python cleanup_fix_dataset.py --input_files a.json b.json --output_path out/ \
        --tasks remove_512 remove_256_javascript remove_512_non_english ftfy_fix_text general_cleaning

Tasks are tried in that order and the first that applies decides the
document (removed, or text rewritten).  Kept documents go to
``<name>_cleaned.json``, removed ones to ``<name>_filtered.json``.
"""
import argparse
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from textclean import fix_text, is_english  # noqa: E402

TASKS = ("remove_512", "remove_256_javascript", "remove_512_non_english", "ftfy_fix_text",
         "general_cleaning")
_SPACES = re.compile(r"  +|\b\n+ |\b\n+")


def process_doc(text, tasks):
    """-> (applied task or None, new text, remove?)."""
    if "remove_512" in tasks and len(text) < 512:
        return "remove_512", text, True
    if "remove_256_javascript" in tasks and len(text) < 256 and "javascript" in text.lower():
        return "remove_256_javascript", text, True
    if "remove_512_non_english" in tasks and len(text) < 512 and not is_english(text):
        return "remove_512_non_english", text, True
    if "ftfy_fix_text" in tasks:
        return "ftfy_fix_text", fix_text(text), False
    if "general_cleaning" in tasks:
        return "general_cleaning", _SPACES.sub(" ", text), False
    return None, text, False


def process_set(tasks, input_file, out_cleaned, out_filtered):
    counts = dict.fromkeys(TASKS, 0)
    with open(input_file, encoding="utf-8") as fin, \
            open(out_cleaned, "w", encoding="utf-8") as fc, \
            open(out_filtered, "w", encoding="utf-8") as ff:
        for line in fin:
            doc = json.loads(line)
            task, text, remove = process_doc(doc["text"], tasks)
            if task:
                counts[task] += 1
            doc["text"] = text
            (ff if remove else fc).write(json.dumps(doc, ensure_ascii=False) + "\n")
    print(f"{input_file}: {counts}", flush=True)
    return counts


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--input_files", nargs="*", required=True)
    p.add_argument("--tasks", nargs="*", required=True, choices=TASKS)
    p.add_argument("--output_path", type=str, default=".")
    p.add_argument("--log_interval", type=int, default=100)
    a = p.parse_args(argv)
    os.makedirs(a.output_path, exist_ok=True)
    out = {}
    for path in a.input_files:
        stem = os.path.splitext(os.path.basename(path))[0]
        out[path] = process_set(a.tasks, path, os.path.join(a.output_path, stem + "_cleaned.json"),
                                os.path.join(a.output_path, stem + "_filtered.json"))
    return out


if __name__ == "__main__":
    main()

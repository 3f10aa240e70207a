"""Concatenate every ``*.json`` (loose json, one document per line) under a
directory (reference ``tools/openwebtext/merge_jsons.py``); lines are
validated as json and copied verbatim."""
import argparse
import glob
import json
import os


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--json_path", type=str, default=".")
    p.add_argument("--output_file", type=str, default="merged_output.json")
    a = p.parse_args(argv)
    files = sorted(glob.glob(os.path.join(a.json_path, "*.json")))
    with open(a.output_file, "w", encoding="utf-8") as out:
        for fname in files:
            with open(fname, encoding="utf-8") as f:
                for row in f:
                    json.loads(row)
                    out.write(row if row.endswith("\n") else row + "\n")
    print(f"merged {len(files)} files into {a.output_file}")


if __name__ == "__main__":
    main()

"""Add ``adlr_id = <prefix>-<10-digit counter>`` to every json line (reference
``tools/openwebtext/add_id.py``)."""
import argparse
import json


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--input_file", type=str, required=True)
    p.add_argument("--output_file", type=str, required=True)
    p.add_argument("--id_prefix", type=str, required=True)
    p.add_argument("--log_interval", type=int, default=100)
    a = p.parse_args(argv)
    with open(a.input_file, encoding="utf-8") as fin, open(a.output_file, "w", encoding="utf-8") as fout:
        n = 0
        for n, line in enumerate(fin, 1):
            d = json.loads(line)
            d["adlr_id"] = f"{a.id_prefix}-{n:010d}"
            fout.write(json.dumps(d, ensure_ascii=False) + "\n")
            if n % a.log_interval == 0:
                print(f"    processed {n} documents", flush=True)
    print(f"done: {n} documents")


if __name__ == "__main__":
    main()

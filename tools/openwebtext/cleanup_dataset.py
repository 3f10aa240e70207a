"""ftfy fix + English filter + drop documents under 128 tokens (reference
``tools/openwebtext/cleanup_dataset.py``).

    python cleanup_dataset.py input.json output.json [--vocab_file V --merge_file M]

Token counts use the framework's GPT-2 BPE when vocab/merge files are given
(the reference downloads GPT-2's), else whitespace words; as in the reference
only documents shorter than 8 * 128 characters are tokenized.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from textclean import fix_text, is_english  # noqa: E402

MIN_DOCUMENT_LENGTH = 128


def _counter(vocab_file, merge_file):
    if vocab_file and merge_file:
        from epfl_megatron_amd.tokenizer.gpt2_bpe import GPT2BPE
        bpe = GPT2BPE(vocab_file, merge_file)
        return lambda t: len(bpe.encode(t))
    return lambda t: len(t.split())


def filter_corpus(filename, out_filename, count_tokens, print_interval=10000):
    st = dict(docs=0, written=0, fixed=0, non_english=0, non_english_chars=0, small=0,
              small_chars=0)
    t0 = time.time()
    with open(filename, encoding="utf-8") as fin, open(out_filename, "w", encoding="utf-8") as f:
        for line in fin:
            st["docs"] += 1
            try:
                doc = json.loads(line)
                text = fix_text(doc["text"])
                st["fixed"] += text != doc["text"]
                doc["text"] = text
                if not is_english(text):
                    st["non_english"] += 1
                    st["non_english_chars"] += len(text)
                    continue
                if len(text) < 8 * MIN_DOCUMENT_LENGTH and count_tokens(text) < MIN_DOCUMENT_LENGTH:
                    st["small"] += 1
                    st["small_chars"] += len(text)
                    continue
                f.write(json.dumps(doc, ensure_ascii=False) + "\n")
                st["written"] += 1
            except (ValueError, KeyError) as e:
                print("    skipping ", line, e)
            if st["docs"] % print_interval == 0:
                print(f"[PROGRESS] {time.time() - t0:.2f} s | {st}", flush=True)
    print(f"[FINAL] {time.time() - t0:.2f} s | {st}", flush=True)
    return st


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("input")
    p.add_argument("output")
    p.add_argument("--vocab_file", default=None)
    p.add_argument("--merge_file", default=None)
    a = p.parse_args(argv)
    return filter_corpus(a.input, a.output, _counter(a.vocab_file, a.merge_file))


if __name__ == "__main__":
    main()

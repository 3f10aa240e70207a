"""Concatenate every indexed dataset of a directory (reference ``tools/merge_datasets.py``).

``--input DIR`` holds ``<name>.bin/<name>.idx`` pairs; they are appended in
sorted name order into ``--output_prefix``.  The output layout (mmap or legacy)
and token dtype follow the first input.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), os.path.pardir)))

from epfl_megatron_amd.data import indexed_dataset  # noqa: E402


def _prefixes(directory):
    names = set()
    for base in os.listdir(directory):
        stem, ext = os.path.splitext(base)
        if ext not in (".bin", ".idx") or not os.path.isfile(os.path.join(directory, base)):
            continue
        other = os.path.join(directory, stem) + (".bin" if ext == ".idx" else ".idx")
        if not os.path.isfile(other):
            raise FileNotFoundError(f"missing {other}")
        names.add(stem)
    return sorted(names)


def main(args):
    builder = None
    for stem in _prefixes(args.input):
        prefix = os.path.join(args.input, stem)
        if builder is None:
            ds = indexed_dataset.make_dataset(prefix, "infer", skip_warmup=True)
            if isinstance(ds, indexed_dataset.MMapIndexedDataset):
                builder = indexed_dataset.MMapIndexedDatasetBuilder(args.output_prefix + ".bin",
                                                                    dtype=ds.dtype)
            else:
                builder = indexed_dataset.IndexedDatasetBuilder(args.output_prefix + ".bin",
                                                                dtype=ds.dtype)
            del ds
        builder.merge_file_(prefix)
    if builder is None:
        raise FileNotFoundError(f"no indexed datasets in {args.input}")
    builder.finalize(args.output_prefix + ".idx")


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--input", type=str, required=True,
                   help="directory containing the .bin/.idx pairs to merge")
    p.add_argument("--output_prefix", type=str, required=True)
    a = p.parse_args(argv)
    if not os.path.isdir(a.input):
        raise NotADirectoryError(a.input)
    if not os.path.isdir(os.path.dirname(os.path.abspath(a.output_prefix))):
        raise NotADirectoryError(os.path.dirname(a.output_prefix))
    return a


if __name__ == "__main__":
    main(parse())

#!/bin/bash
# Tokenize a train and a validation split (see README.md).  Override any of the
# variables from the environment.
set -euo pipefail
REPO=${REPO:-/workspace}
DATA=${DATA:-/data}
TOKENIZER_TYPE=${TOKENIZER_TYPE:-FalconTokenizer}
VOCAB=${VOCAB:-$DATA/tokenizer.json}
WORKERS=${WORKERS:-16}
cd "$REPO"
python __graft_entry__.py build
for split in train valid; do
  python tools/preprocess_data.py --input "$DATA/$split.jsonl" --output_prefix "$DATA/wiki-$split" \
    --dataset_impl mmap --tokenizer_type "$TOKENIZER_TYPE" --vocab_file "$VOCAB" \
    --workers "$WORKERS" --chunk_size 2048 --append_eod
done

#!/bin/bash
# jsonl -> indexed corpus.  Usage: examples/preprocess.sh INPUT.jsonl OUT_PREFIX TOKENIZER_MODEL
set -e
python "$(dirname "$0")/../tools/preprocess_data.py" --input $1 --output_prefix $2 \
  --tokenizer_type SentencePieceTokenizer --vocab_file $3 --append_eod \
  --workers 16 --chunk_size 32

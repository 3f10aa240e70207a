#!/bin/bash
# Meta / Hugging Face weights (local directory) -> Megatron release checkpoint.
# Usage: examples/weights2megatron.sh <llama|llama2|codellama|falcon> SIZE WEIGHTS_DIR OUT_DIR
set -e
python "$(dirname "$0")/../weights2megatron/weights2megatron.py" $1 --size $2 \
  --cache-dir $3 --out $4

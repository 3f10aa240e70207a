#!/bin/bash
# Re-shard a checkpoint to TP x PP (reference examples/parallelize.sh).
# Usage: examples/parallelize.sh <llama|llama2|falcon|gpt> IN_DIR OUT_DIR TP PP [VOCAB_FILE]
set -e
MODEL=$1; IN=$2; OUT=$3; TP=$4; PP=$5; VOCAB=$6
EXTRA=""; [[ -n $VOCAB ]] && EXTRA="--vocab_file $VOCAB"
python "$(dirname "$0")/../tools/checkpoint_util.py" --model_type $MODEL --load_dir $IN \
  --save_dir $OUT --target_tensor_parallel_size $TP --target_pipeline_parallel_size $PP $EXTRA

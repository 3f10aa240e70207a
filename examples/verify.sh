#!/bin/bash
# Compare a (TP=PP=1) Megatron checkpoint against its Hugging Face model on real data.
# Usage: examples/verify.sh <llama|llama2|falcon> MEGATRON_DIR HF_DIR DATA_PREFIX [VOCAB]
set -e
MODEL=$1; CKPT=$2; HF=$3; DATA=$4; VOCAB=$5
TOK=SentencePieceTokenizer; [[ $MODEL == falcon ]] && TOK=FalconTokenizer
EXTRA=""; [[ -n $VOCAB ]] && EXTRA="--vocab_file $VOCAB"
python -m torch.distributed.run --nproc_per_node 1 --master_addr 127.0.0.1 \
  "$(dirname "$0")/../verify_correctness.py" --model_name $MODEL --load $CKPT \
  --huggingface_cache $HF --data_path $DATA --tokenizer_type $TOK $EXTRA --bf16

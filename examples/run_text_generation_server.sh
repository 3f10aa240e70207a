#!/bin/bash
# Serve a checkpoint over REST (PUT /api).  Usage: examples/run_text_generation_server.sh
#   <llama2|falcon|gpt> CKPT_DIR TOKENIZER [TP] [PORT]
set -e
MODEL=$1; CKPT=$2; VOCAB=$3; TP=${4:-1}; PORT=${5:-5000}
TOK=SentencePieceTokenizer; [[ $MODEL == falcon ]] && TOK=FalconTokenizer
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -m torch.distributed.run --nproc_per_node $TP --master_addr 127.0.0.1 \
  "$(dirname "$0")/../tools/run_text_generation_server.py" --model_name $MODEL --load $CKPT \
  --use_checkpoint_args --tokenizer_type $TOK --vocab_file $VOCAB --bf16 --use_flash_attn \
  --tensor_model_parallel_size $TP --micro_batch_size 1 --port $PORT

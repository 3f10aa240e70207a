#!/bin/bash
# Zero-shot evaluation of a (sharded) checkpoint on WikiText-103 or LAMBADA.
#   TASK=WIKITEXT103 DATA=wiki.test.tokens CKPT=/ckpt/llama2-7b-tp1 ./examples/evaluate_zeroshot.sh
#   TASK=LAMBADA DATA=lambada_test.jsonl ... (add --strict_lambada for whole-word targets)
set -e
NGPU=${NGPU:-1}; TP=${TP:-1}; PP=${PP:-1}
TASK=${TASK:-WIKITEXT103}
torchrun --nproc-per-node "$NGPU" --master-addr 127.0.0.1 --master-port ${PORT:-29500} \
  tasks/main.py --task "$TASK" --valid_data "$DATA" --load "$CKPT" \
  --model_name ${MODEL:-llama2} --tokenizer_type SentencePieceTokenizer \
  --vocab_file "${TOKENIZER:-$CKPT/tokenizer.model}" \
  --tensor_model_parallel_size $TP --pipeline_model_parallel_size $PP \
  --use_checkpoint_args --no_load_optim --no_load_rng --bf16 \
  --micro_batch_size ${MBS:-8} --overlapping_eval ${OVERLAP:-32} --log_interval 10 "$@"

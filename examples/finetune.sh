#!/bin/bash
# Fine-tune GPT / Llama / Llama-2 / Falcon on one MI355X node (8 GPUs, RCCL over xGMI).
# Same flags as the reference (examples/finetune.sh); MI355X defaults differ:
#   * TP=1 by default: a 7B/13B model + fp32 master + Adam state fits in 288 GB HBM,
#     so pure data parallelism (distributed optimizer) avoids TP all-reduces on xGMI;
#   * no CUDA_DEVICE_MAX_CONNECTIONS (ordering comes from HIP events).
# Usage: examples/finetune.sh <gpt|llama|llama2|falcon> [--size 7] [--tp 1] [--pp 1]
#        [--gpus 8] [--micro-batch 4] [--global-batch 512] [--data PREFIX] [--load DIR]
#        [--save DIR] [--vocab FILE] [--wandb] [--synthetic]
set -e
MODEL=$1; shift || true
SIZE=7; TP=1; PP=1; GPUS=8; MBS=4; GBS=512; DATA=""; LOAD=""; SAVE="";
VOCAB=""; WANDB=0; SYNTH=0
while [[ $# -gt 0 ]]; do
  case $1 in
    --size) SIZE=$2; shift 2;; --tp) TP=$2; shift 2;; --pp) PP=$2; shift 2;;
    --gpus) GPUS=$2; shift 2;; --micro-batch) MBS=$2; shift 2;;
    --global-batch) GBS=$2; shift 2;; --data) DATA=$2; shift 2;; --load) LOAD=$2; shift 2;;
    --save) SAVE=$2; shift 2;; --vocab) VOCAB=$2; shift 2;; --wandb) WANDB=1; shift;;
    --synthetic) SYNTH=1; shift;;
    *) echo "unknown argument $1"; exit 1;;
  esac
done
LR=3e-4
case $MODEL in
  falcon) TOK=FalconTokenizer; SEQ=2048; EXTRA="--parallel_attn";;
  llama|llama2)
    TOK=SentencePieceTokenizer
    EXTRA="--use_rms_norm --glu_activation swiglu --no_tie_embed_logits"
    [[ -n $VOCAB ]] && EXTRA="$EXTRA --vocab_file $VOCAB"
    if [[ $MODEL == llama ]]; then SEQ=2048; EXTRA="$EXTRA --layernorm_epsilon 1e-6"
    else SEQ=4096; EXTRA="$EXTRA --layernorm_epsilon 1e-5"; (( SIZE > 13 )) && LR=1.5e-4; fi;;
  gpt) TOK=GPT2BPETokenizer; SEQ=2048
       EXTRA="--num_layers 4 --hidden_size 512 --num_attention_heads 8";;
  *) echo "model must be gpt, llama, llama2 or falcon"; exit 1;;
esac
ARGS="--model_name $MODEL --tokenizer_type $TOK --tensor_model_parallel_size $TP
  --pipeline_model_parallel_size $PP --micro_batch_size $MBS --global_batch_size $GBS
  --seq_length $SEQ --max_position_embeddings $SEQ --use_flash_attn --bf16
  --position_embedding_type rotary --hidden_dropout 0.0 --attention_dropout 0.0
  --no_bias_gelu_fusion --no_bias_dropout_fusion --adam_beta1 0.9 --adam_beta2 0.95
  --adam_eps 1e-5 --lr_decay_style cosine --lr_warmup_iters 2000 --lr $LR --min_lr 1e-6
  --weight_decay 0.1 --train_iters 10000 --log_interval 1 --save_interval 500
  --eval_interval 500 --eval_iters 10 --use_distributed_optimizer
  --recompute_granularity selective $EXTRA"
(( TP > 1 )) && ARGS="$ARGS --sequence_parallel"
[[ -n $LOAD ]] && ARGS="$ARGS --load $LOAD --use_checkpoint_args"
[[ -n $SAVE ]] && ARGS="$ARGS --save $SAVE"
[[ $WANDB == 1 ]] && ARGS="$ARGS --wandb_logger"
if [[ $SYNTH == 1 ]]; then ARGS="$ARGS --synthetic_data"; else ARGS="$ARGS --data_path $DATA"; fi
export HSA_ENABLE_IPC_MODE_LEGACY=0
exec python -m torch.distributed.run --nproc_per_node $GPUS --nnodes 1 \
  --master_addr 127.0.0.1 --master_port 6000 "$(dirname "$0")/../finetune.py" $ARGS

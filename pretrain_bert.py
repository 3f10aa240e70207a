"""Pretrain BERT (masked LM + sentence-order prediction) — reference
``pretrain_bert.py``.  Corpus: ``tools/preprocess_data.py --split_sentences``."""
from functools import partial

import torch
import torch.nn.functional as F

from epfl_megatron_amd import get_args, get_timers, print_rank_0
from epfl_megatron_amd.data.dataset_utils import build_train_valid_test_datasets
from epfl_megatron_amd.initialize import initialize_megatron
from epfl_megatron_amd.models import BertModel, ModelType
from epfl_megatron_amd.parallel import tensor as tensor_parallel
from epfl_megatron_amd.training import pretrain
from epfl_megatron_amd.utils.misc import average_losses_across_data_parallel_group


def model_provider(pre_process=True, post_process=True):
    print_rank_0("building BERT model ...")
    args = get_args()
    return BertModel(num_tokentypes=2 if args.bert_binary_head else 0,
                     add_binary_head=args.bert_binary_head, parallel_output=True,
                     pre_process=pre_process, post_process=post_process,
                     model_type=ModelType.encoder_or_decoder)


def get_batch(data_iterator):
    keys = ["text", "types", "labels", "is_random", "loss_mask", "padding_mask"]
    data = next(data_iterator) if data_iterator is not None else None
    b = tensor_parallel.broadcast_data(keys, data, torch.int64)
    return (b["text"].long(), b["types"].long(), b["is_random"].long(),
            b["loss_mask"].float(), b["labels"].long(), b["padding_mask"].long())


def loss_func(loss_mask, sentence_order, output_tensor):
    lm_loss_, sop_logits = output_tensor
    loss_mask = loss_mask.float()
    lm_loss = torch.sum(lm_loss_.float().view(-1) * loss_mask.reshape(-1)) / loss_mask.sum()
    if sop_logits is None:
        avg = average_losses_across_data_parallel_group([lm_loss])
        return lm_loss, {"lm loss": avg[0]}
    sop_loss = F.cross_entropy(sop_logits.view(-1, 2).float(), sentence_order.view(-1),
                               ignore_index=-1)
    avg = average_losses_across_data_parallel_group([lm_loss, sop_loss])
    return lm_loss + sop_loss, {"lm loss": avg[0], "sop loss": avg[1]}


def forward_step(data_iterator, model):
    args = get_args()
    timers = get_timers()
    timers("batch-generator", log_level=2).start()
    tokens, types, sentence_order, loss_mask, lm_labels, padding_mask = get_batch(data_iterator)
    timers("batch-generator").stop()
    if not args.bert_binary_head:
        types = None
    out = model(tokens, padding_mask, tokentype_ids=types, lm_labels=lm_labels)
    return out, partial(loss_func, loss_mask, sentence_order)


def train_valid_test_datasets_provider(train_val_test_num_samples):
    args = get_args()
    print_rank_0("> building train, validation, and test datasets for BERT ...")
    ds = build_train_valid_test_datasets(
        data_prefix=args.data_path, data_impl=args.data_impl, splits_string=args.split,
        train_valid_test_num_samples=train_val_test_num_samples, max_seq_length=args.seq_length,
        masked_lm_prob=args.mask_prob, short_seq_prob=args.short_seq_prob, seed=args.seed,
        skip_warmup=(not args.mmap_warmup), binary_head=args.bert_binary_head)
    print_rank_0("> finished creating BERT datasets ...")
    return ds


def main(args_list=None):
    initialize_megatron(None, {"tokenizer_type": "BertWordPieceLowerCase"}, args_list=args_list)
    return pretrain(get_args(), train_valid_test_datasets_provider, model_provider,
                    ModelType.encoder_or_decoder, forward_step)


if __name__ == "__main__":
    main()

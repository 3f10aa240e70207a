"""Pretrain T5 (span corruption) — reference ``pretrain_t5.py``.
Needs ``--encoder_seq_length``, ``--decoder_seq_length`` and ``--vocab_extra_ids``."""
from functools import partial

import torch

from epfl_megatron_amd import get_args, get_timers, print_rank_0
from epfl_megatron_amd.data.dataset_utils import build_train_valid_test_datasets
from epfl_megatron_amd.initialize import initialize_megatron
from epfl_megatron_amd.models import ModelType, T5Model
from epfl_megatron_amd.parallel import tensor as tensor_parallel
from epfl_megatron_amd.training import pretrain
from epfl_megatron_amd.utils.misc import average_losses_across_data_parallel_group


def model_provider(pre_process=True, post_process=True, add_encoder=True, add_decoder=True):
    print_rank_0("building T5 model ...")
    return T5Model(num_tokentypes=0, parallel_output=True, pre_process=pre_process,
                   post_process=post_process, add_encoder=add_encoder, add_decoder=add_decoder,
                   model_type=ModelType.encoder_and_decoder)


def get_batch(data_iterator):
    keys = ["text_enc", "text_dec", "labels", "loss_mask", "enc_mask", "dec_mask",
            "enc_dec_mask"]
    data = next(data_iterator) if data_iterator is not None else None
    b = tensor_parallel.broadcast_data(keys, data, torch.int64)
    # masks: dataset 1 = keep -> attention kernels' True = masked
    return (b["text_enc"].long(), b["text_dec"].long(), b["loss_mask"].float(),
            b["labels"].long(), b["enc_mask"] < 0.5, b["dec_mask"] < 0.5,
            b["enc_dec_mask"] < 0.5)


def loss_func(loss_mask, output_tensor):
    lm_loss = torch.sum(output_tensor.float().view(-1) * loss_mask.reshape(-1)) / loss_mask.sum()
    avg = average_losses_across_data_parallel_group([lm_loss])
    return lm_loss, {"lm loss": avg[0]}


def forward_step(data_iterator, model):
    timers = get_timers()
    timers("batch generator", log_level=2).start()
    enc, dec, loss_mask, labels, enc_mask, dec_mask, enc_dec_mask = get_batch(data_iterator)
    timers("batch generator").stop()
    out = model(enc, dec, enc_mask, dec_mask, enc_dec_mask, tokentype_ids=None, lm_labels=labels)
    return out, partial(loss_func, loss_mask)


def train_valid_test_datasets_provider(train_val_test_num_samples):
    args = get_args()
    print_rank_0("> building train, validation, and test datasets for T5 ...")
    ds = build_train_valid_test_datasets(
        data_prefix=args.data_path, data_impl=args.data_impl, splits_string=args.split,
        train_valid_test_num_samples=train_val_test_num_samples,
        max_seq_length=args.encoder_seq_length, max_seq_length_dec=args.decoder_seq_length,
        masked_lm_prob=args.mask_prob, short_seq_prob=args.short_seq_prob, seed=args.seed,
        skip_warmup=(not args.mmap_warmup), dataset_type="t5")
    print_rank_0("> finished creating T5 datasets ...")
    return ds


def main(args_list=None):
    initialize_megatron(None, {"tokenizer_type": "BertWordPieceLowerCase"}, args_list=args_list)
    return pretrain(get_args(), train_valid_test_datasets_provider, model_provider,
                    ModelType.encoder_and_decoder, forward_step)


if __name__ == "__main__":
    main()

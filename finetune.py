"""Fine-tune / pretrain GPT, Llama-1/2 or Falcon (reference ``finetune.py``).

Public API kept: ``model_provider``, ``get_batch``, ``loss_func``,
``forward_step``, ``train_valid_test_datasets_provider``, ``extra_args`` and
the underscore-style CLI.  ``--synthetic_data`` (MI355X addition) trains on
deterministic synthetic tokens without a corpus.
"""
import datetime as dt
from functools import partial

import torch

from epfl_megatron_amd import get_args, get_tokenizer, get_timers, print_rank_0
from epfl_megatron_amd.initialize import initialize_megatron
from epfl_megatron_amd.models import FalconModel, GPTModel, LlamaModel, ModelType
from epfl_megatron_amd.parallel import tensor as tensor_parallel
from epfl_megatron_amd.parallel.context import cp_token_mean, get_batch_on_this_cp_rank
from epfl_megatron_amd.training import pretrain
from epfl_megatron_amd.utils.misc import (average_losses_across_data_parallel_group, doc_bounds,
                                          get_ltor_masks_and_position_ids)


def model_provider(pre_process=True, post_process=True):
    print_rank_0("Building model ...")
    args = get_args()
    name = args.model_name
    if name == "gpt":
        cls = GPTModel
    elif name == "falcon":
        cls = FalconModel
    elif name in ("llama", "llama2"):
        cls = partial(LlamaModel, version=1 if name == "llama" else 2)
    else:
        raise KeyError(f"Unknown model {name}")
    if isinstance(args.model_type, ModelType):
        model_type = args.model_type
    else:
        model_type = ModelType[args.model_type]
    return cls(num_tokentypes=0, parallel_output=True, pre_process=pre_process,
               post_process=post_process, model_type=model_type)


def get_batch(data_iterator):
    args = get_args()
    tokenizer = get_tokenizer()
    keys = ["text"]
    data = next(data_iterator) if data_iterator is not None else None
    if data is not None and not torch.is_tensor(data["text"]):
        data = {"text": torch.as_tensor(data["text"])}
    data_b = tensor_parallel.broadcast_data(keys, data, torch.int64)
    tokens_ = data_b["text"].long()
    labels = tokens_[:, 1:].contiguous()
    tokens = tokens_[:, :-1].contiguous()
    attention_mask, loss_mask, position_ids = get_ltor_masks_and_position_ids(
        tokens, tokenizer.eod, args.reset_position_ids, args.reset_attention_mask,
        args.eod_mask_loss, flash_doc_bounds=args.use_flash_attn)
    if args.context_parallel_size > 1:
        # this rank's sequence chunk; the causal mask is implied by the ring,
        # packed documents travel as the WHOLE sequence's int32 [2, b, S] bounds
        tokens, labels, loss_mask, position_ids = get_batch_on_this_cp_rank(
            [tokens, labels, loss_mask, position_ids])
        attention_mask = doc_bounds(data_b["text"].long()[:, :-1], tokenizer.eod) \
            if args.reset_attention_mask else None
    return tokens, labels, loss_mask, attention_mask, position_ids


def loss_func(loss_mask, output_tensor):
    losses = output_tensor.float()
    loss_mask = loss_mask.view(-1).float()
    loss = cp_token_mean(losses.view(-1), loss_mask)
    averaged = average_losses_across_data_parallel_group([loss])
    return loss, {"lm loss": averaged[0]}


def forward_step(data_iterator, model):
    timers = get_timers()
    timers("batch-generator", log_level=2).start()
    tokens, labels, loss_mask, attention_mask, position_ids = get_batch(data_iterator)
    timers("batch-generator").stop()
    args = get_args()
    # RoPE position ids are only needed when they are not arange(s).
    pos = position_ids if (args.reset_position_ids or args.context_parallel_size > 1) else None
    if args.position_embedding_type.name == "absolute":
        pos = position_ids
    output_tensor = model(tokens, pos, attention_mask, labels=labels)
    return output_tensor, partial(loss_func, loss_mask)


def train_valid_test_datasets_provider(train_val_test_num_samples):
    args = get_args()
    if args.synthetic_data:
        from epfl_megatron_amd.data.synthetic import synthetic_train_valid_test_datasets
        print_rank_0("> building synthetic train, validation, and test datasets ...")
        vocab = get_tokenizer().vocab_size
        return synthetic_train_valid_test_datasets(train_val_test_num_samples, args.seq_length,
                                                   vocab, args.seed,
                                                   pattern=args.synthetic_pattern)
    from epfl_megatron_amd.data.gpt_dataset import build_train_valid_test_datasets
    print_rank_0("> building train, validation, and test datasets for GPT ...")
    train_ds, valid_ds, test_ds = build_train_valid_test_datasets(
        data_prefix=args.data_path, data_impl=args.data_impl, splits_string=args.split,
        train_valid_test_num_samples=train_val_test_num_samples, seq_length=args.seq_length,
        seed=args.seed, skip_warmup=(not args.mmap_warmup),
        train_data_prefix=args.train_data_path, valid_data_prefix=args.valid_data_path,
        test_data_prefix=args.test_data_path)
    print_rank_0("> finished creating GPT datasets ...")
    return train_ds, valid_ds, test_ds


def extra_args(parser):
    group = parser.add_argument_group(title="validation set")
    group.add_argument("--model_name", choices={"gpt", "llama", "falcon", "llama2"},
                       default="gpt")
    group.add_argument("--model_type", choices={"encoder_or_decoder", "encoder_and_decoder"},
                       default="encoder_or_decoder")
    group.add_argument("--log_learning_rate_to_tensorboard", type=bool, default=True)
    group.add_argument("--log_loss_scale_to_tensorboard", type=bool, default=True)
    return parser


def main(args_list=None):
    initialize_megatron(extra_args, {"tokenizer_type": "GPT2BPETokenizer"}, args_list=args_list)
    args = get_args()
    out = pretrain(args, train_valid_test_datasets_provider, model_provider,
                   ModelType.encoder_or_decoder, forward_step)
    print(f"Done {dt.datetime.now(dt.timezone.utc)}")
    return out


if __name__ == "__main__":
    main()

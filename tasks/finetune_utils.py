"""Epoch-based finetuning driver shared by GLUE / RACE / retriever tasks
(reference ``tasks/finetune_utils.py:24-309``).

Differences from the language-model ``pretrain()`` loop: data comes from a
``DistributedSampler`` over the DP group (one epoch = one pass), the batch is
a dict of padded ``[CLS] a [SEP] b`` samples, and an optional per-epoch
callback computes accuracies.  Gradient accumulation is not supported
(``num_microbatches == 1``), exactly as in the reference.
"""
import sys
from functools import partial

import torch

from epfl_megatron_amd import get_args, get_num_microbatches, get_timers, print_rank_0
from epfl_megatron_amd import training
from epfl_megatron_amd.checkpointing import load_checkpoint, save_checkpoint
from epfl_megatron_amd.models import ModelType
from epfl_megatron_amd.parallel import state
from epfl_megatron_amd.utils.misc import average_losses_across_data_parallel_group


def _device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")


def process_batch(batch, is_fp16=False):
    """Batch dict -> (tokens, types, labels, padding mask) on the compute device."""
    dev = _device()
    tokens = torch.as_tensor(batch["text"]).long().to(dev, non_blocking=True).contiguous()
    types = torch.as_tensor(batch["types"]).long().to(dev, non_blocking=True).contiguous()
    labels = torch.as_tensor(batch["label"]).long().to(dev, non_blocking=True).contiguous()
    mask = torch.as_tensor(batch["padding_mask"]).to(dev, non_blocking=True)
    mask = mask.to(torch.half if is_fp16 else torch.float).contiguous()
    return tokens, types, labels, mask


def _next_batch(batch):
    """The schedules hand either an iterator or an already materialised batch."""
    if isinstance(batch, dict):
        return batch
    try:
        return next(batch)
    except TypeError:
        return batch


def cross_entropy_loss_func(labels, output_tensor):
    loss = torch.nn.functional.cross_entropy(output_tensor.contiguous().float(), labels)
    averaged = average_losses_across_data_parallel_group([loss])
    return loss, {"lm loss": averaged[0]}


def _cross_entropy_forward_step(batch, model):
    args = get_args()
    timers = get_timers()
    timers("batch-generator", log_level=2).start()
    tokens, types, labels, mask = process_batch(_next_batch(batch), args.fp16)
    timers("batch-generator").stop()
    return model(tokens, mask, tokentype_ids=types), partial(cross_entropy_loss_func, labels)


def build_data_loader(dataset, micro_batch_size, num_workers, drop_last, task_collate_fn=None):
    """Per-rank loader: each DP rank reads a disjoint shard of every epoch."""
    sampler = torch.utils.data.distributed.DistributedSampler(
        dataset, num_replicas=state.get_data_parallel_world_size(),
        rank=state.get_data_parallel_rank())
    return torch.utils.data.DataLoader(dataset, batch_size=micro_batch_size, sampler=sampler,
                                       shuffle=False, num_workers=num_workers,
                                       drop_last=drop_last, pin_memory=torch.cuda.is_available(),
                                       collate_fn=task_collate_fn)


def _build_infinite_size_dataloader(dataloader):
    while True:
        yield from dataloader


def _build_train_valid_dataloaders(train_dataset, valid_dataset, task_collate_fn=None):
    args = get_args()
    print_rank_0("building train and validation dataloaders ...")
    train_dl = build_data_loader(train_dataset, args.micro_batch_size, args.num_workers,
                                 not args.keep_last, task_collate_fn)
    args.train_iters_per_epoch = len(train_dl)
    args.train_iters = args.epochs * args.train_iters_per_epoch
    valid_dl = _build_infinite_size_dataloader(
        build_data_loader(valid_dataset, args.micro_batch_size, args.num_workers,
                          not args.keep_last, task_collate_fn))
    # A "sample" of a multiple-choice dataset expands into sample_multiplier
    # rows of the batch dimension; pipeline shapes and the sample-based LR
    # schedule must see the expanded size.
    args.orig_micro_batch_size = args.micro_batch_size
    args.orig_global_batch_size = args.global_batch_size
    mult = getattr(train_dataset, "sample_multiplier", 1)
    args.micro_batch_size *= mult
    args.global_batch_size *= mult
    return train_dl, valid_dl


def _train(model, optimizer, opt_param_scheduler, forward_step, train_dataloader,
           valid_dataloader, end_of_epoch_callback, args):
    timers = get_timers()
    assert get_num_microbatches() == 1, \
        "finetuning with gradient accumulation is not supported"
    for m in model:
        m.train()
    losses_dict_sum = {}
    start_epoch = args.iteration // args.train_iters_per_epoch
    skip = args.iteration % args.train_iters_per_epoch
    iteration = args.iteration
    report_memory_flag = True
    timers("interval-time", log_level=0).start(barrier=True)
    for epoch in range(start_epoch, args.epochs):
        print_rank_0(f"working on epoch {epoch + 1} ...")
        train_dataloader.sampler.set_epoch(args.seed + epoch)
        for i, batch in enumerate(train_dataloader):
            if i < skip:
                continue
            skip = 0
            losses, skipped, grad_norm, nz = training.train_step(
                forward_step, batch, model, optimizer, opt_param_scheduler, args)
            iteration += 1
            args.consumed_train_samples += args.global_batch_size
            params_norm = None
            if args.log_params_norm:
                from epfl_megatron_amd.utils.misc import calc_params_l2_norm
                params_norm = calc_params_l2_norm(model)
            report_memory_flag = training.training_log(
                losses, losses_dict_sum, optimizer.param_groups[0]["lr"], iteration,
                float(optimizer.get_loss_scale()), skipped, grad_norm, params_norm, nz,
                report_memory_flag=report_memory_flag)
            saved = False
            if args.save and args.save_interval and iteration % args.save_interval == 0:
                save_checkpoint(iteration, model, optimizer, opt_param_scheduler)
                saved = True
            if args.eval_interval and iteration % args.eval_interval == 0:
                training.evaluate_and_print_results(f"iteration {iteration}", forward_step,
                                                    valid_dataloader, model, iteration, None,
                                                    False, args=args)
            if args.exit_interval and iteration % args.exit_interval == 0:
                if not saved and args.save:
                    save_checkpoint(iteration, model, optimizer, opt_param_scheduler)
                if torch.distributed.is_initialized():
                    torch.distributed.barrier()
                print_rank_0(f"exiting program at iteration {iteration}")
                sys.exit()
        if args.save:
            save_checkpoint(iteration, model, optimizer, opt_param_scheduler)
        if end_of_epoch_callback is not None:
            end_of_epoch_callback(model, epoch)
    args.iteration = iteration


def finetune(train_valid_datasets_provider, model_provider,
             model_type=ModelType.encoder_or_decoder, forward_step=_cross_entropy_forward_step,
             end_of_epoch_callback_provider=None, task_collate_fn=None):
    """Build data/model/optimizer, optionally load ``--pretrained_checkpoint``
    (model weights only, no RNG), then train ``--epochs`` epochs or, with
    ``--epochs 0``, just run the end-of-epoch metrics in prediction mode."""
    args = get_args()
    timers = get_timers()
    assert args.rampup_batch_size is None, "batch size ramp-up is not supported for finetuning"
    timers("train/valid/test dataset/dataloder", log_level=0).start()
    if args.epochs > 0:
        train_ds, valid_ds = train_valid_datasets_provider()
        train_dl, valid_dl = _build_train_valid_dataloaders(train_ds, valid_ds, task_collate_fn)
    else:
        args.train_iters = 0
        args.orig_micro_batch_size = args.micro_batch_size
        args.orig_global_batch_size = args.global_batch_size
    timers("train/valid/test dataset/dataloder").stop()

    timers("callback function", log_level=0).start()
    callback = end_of_epoch_callback_provider() if end_of_epoch_callback_provider else None
    timers("callback function").stop()

    timers("model and optimizer", log_level=0).start()
    model, optimizer, sched = training._setup_model_and_optimizer(model_provider, model_type,
                                                                  args=args)
    timers("model and optimizer").stop()

    timers("pretrained checkpoint", log_level=0).start(barrier=True)
    if args.iteration == 0 and args.pretrained_checkpoint is not None:
        saved_load, saved_rng = args.load, args.no_load_rng
        args.load, args.no_load_rng = args.pretrained_checkpoint, True
        load_checkpoint(model, None, None)
        args.load, args.no_load_rng = saved_load, saved_rng
        optimizer.reload_model_params()  # master fp32 copies follow the loaded weights
    timers("pretrained checkpoint").stop()
    print_rank_0("done with setups ...")
    timers.log(["train/valid/test dataset/dataloder", "callback function",
                "model and optimizer", "pretrained checkpoint"], barrier=True)
    print_rank_0("training ...")
    if args.epochs > 0:
        _train(model, optimizer, sched, forward_step, train_dl, valid_dl, callback, args)
    elif callback is not None:
        print_rank_0("evaluation only mode, setting epoch to -1")
        callback(model, epoch=-1, output_predictions=True)
    print_rank_0("done :-)")
    return model

"""Accuracy evaluation for the classification / multiple-choice tasks
(reference ``tasks/eval_utils.py:18-181``).

``accuracy_func_provider`` returns the end-of-epoch callback: a forward-only
pass over each ``--valid_data`` file through the pipeline schedule, argmax of
the logits, and a DP all-reduce of ``[correct, total]`` on the last stage.
With ``output_predictions`` (evaluation-only mode, DP=1) the softmaxes,
labels and uids are saved next to ``--load`` as ``predictions_<names>.pt``.
"""
import os
import time
from functools import partial

import torch

from epfl_megatron_amd import get_args, is_last_rank, print_rank_last
from epfl_megatron_amd.parallel import state
from epfl_megatron_amd.parallel.pipeline.schedules import get_forward_backward_func

from . import finetune_utils


def accuracy_func_provider(single_dataset_provider):
    args = get_args()
    loaders = []
    for path in args.valid_data:
        ds = single_dataset_provider(path)
        dl = finetune_utils.build_data_loader(
            ds, args.orig_micro_batch_size, num_workers=args.num_workers,
            drop_last=state.get_data_parallel_world_size() > 1)
        loaders.append((ds.dataset_name, dl))

    def metrics_func(model, epoch, output_predictions=False):
        print_rank_last("calculating metrics ...")
        correct = total = 0
        named, names = [], "predictions"
        if output_predictions:
            assert state.get_data_parallel_world_size() == 1
        for name, dl in loaders:
            out = calculate_correct_answers(name, model, dl, epoch, output_predictions)
            correct += out[0]
            total += out[1]
            if output_predictions:
                named.append((name, out[2]))
                names += "_" + name
        if is_last_rank() and total > 0:
            print(f" >> |epoch: {epoch}| overall: correct / total = {correct} / {total} = "
                  f"{100.0 * correct / total:.4f} %", flush=True)
        if output_predictions and is_last_rank():
            assert args.load is not None
            torch.save(named, os.path.join(args.load, names + ".pt"))
        return correct, total

    return metrics_func


def calculate_correct_answers(name, model, dataloader, epoch, output_predictions):
    """Returns ``(correct, total[, (softmaxes, labels, uids)])`` reduced over DP
    (zeros on non-last pipeline stages)."""
    args = get_args()
    fwd_bwd = get_forward_backward_func()
    t0 = time.time()
    for m in model:
        m.eval()
    saved_mbs, saved_gbs = args.micro_batch_size, args.global_batch_size
    mult = getattr(dataloader.dataset, "sample_multiplier", 1)
    num_micro = args.orig_global_batch_size // (args.orig_micro_batch_size *
                                                args.data_parallel_size)

    def loss_func(batch, labels, logits):
        pred = torch.argmax(logits, dim=-1)
        d = {"total": labels.size(0), "correct": int((pred == labels).sum())}
        if output_predictions:
            d["softmaxes"] = torch.softmax(logits.float(), -1).cpu().tolist()
            d["labels"] = labels.cpu().tolist()
            d["ids"] = torch.as_tensor(batch["uid"]).tolist()
        return 0, d

    def fwd(batch, model):
        b = finetune_utils._next_batch(batch)
        tokens, types, labels, mask = finetune_utils.process_batch(b, args.fp16)
        return model(tokens, mask, tokentype_ids=types), partial(loss_func, b, labels)

    correct = total = 0
    soft, labs, ids = [], [], []
    with torch.no_grad():
        for batch in dataloader:
            # drop_last may be off in eval-only mode: size the pipeline
            # transfers for the actual (possibly short) batch.
            n = len(batch["label"])
            args.micro_batch_size = n * mult
            args.global_batch_size = n * mult * num_micro
            for d in fwd_bwd(fwd, batch, model, optimizer=None, timers=None, forward_only=True):
                total += d["total"]
                correct += d["correct"]
                if output_predictions:
                    soft += d["softmaxes"]
                    labs += d["labels"]
                    ids += d["ids"]
    for m in model:
        m.train()
    args.micro_batch_size, args.global_batch_size = saved_mbs, saved_gbs

    if not state.is_pipeline_last_stage():
        return (0, 0, ()) if output_predictions else (0, 0)
    red = torch.tensor([correct, total], dtype=torch.long, device=finetune_utils._device())
    if torch.distributed.is_initialized():
        torch.distributed.all_reduce(red, group=state.get_data_parallel_group())
    correct, total = int(red[0]), int(red[1])
    if total:
        print_rank_last(f" > |epoch: {epoch}| metrics for {name}: correct / total = {correct} / "
                        f"{total} = {100.0 * correct / total:.4f} %, elapsed time (sec): "
                        f"{time.time() - t0:.3f}")
    if output_predictions:
        return correct, total, (soft, labs, ids)
    return correct, total

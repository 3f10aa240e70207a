"""Supervised retriever validation (reference ``tasks/orqa/supervised/eval_utils.py``):
for every validation question, rank its positive passage among the batch's
positives plus the per-question negatives; report the mean rank and top-k
accuracies averaged over DP."""
import math
import time

import numpy as np
import torch

from epfl_megatron_amd import get_args, print_rank_0
from epfl_megatron_amd.parallel import state
from epfl_megatron_amd.utils.misc import average_losses_across_data_parallel_group

from ... import finetune_utils

_LONG_KEYS = ("query", "query_mask", "query_types", "query_pad_mask", "context", "context_mask",
              "context_types", "context_pad_mask")


def task_collate_fn(batch_data):
    out = {k: [d[k] for d in batch_data] for k in batch_data[0]}
    for k in _LONG_KEYS:
        out[k] = torch.as_tensor(np.stack(out[k]), dtype=torch.long)
    if "neg_context" in out:  # negatives of all questions, flattened along dim 0
        for k in ("neg_context", "neg_context_mask", "neg_context_types"):
            out[k] = torch.as_tensor(np.concatenate(out[k]), dtype=torch.long)
    return out


def process_batch(batch):
    dev = finetune_utils._device()

    def long(k):
        return batch[k].long().to(dev)

    def mask(k):
        return (batch[k] < 0.5).to(dev)
    neg = (long("neg_context"), mask("neg_context_mask"), long("neg_context_types")) \
        if "neg_context" in batch else (None, None, None)
    return (long("query"), mask("query_mask"), long("query_types"), long("query_pad_mask"),
            long("context"), mask("context_mask"), long("context_types"),
            long("context_pad_mask"), *neg, batch["reference"])


def accuracy_func_provider(single_dataset_provider, rank0sampler=False):
    args = get_args()
    dataset = single_dataset_provider(args.valid_data)
    drop_last = state.get_data_parallel_world_size() > 1 and not rank0sampler
    dataloader = finetune_utils.build_data_loader(
        dataset, args.eval_micro_batch_size or args.micro_batch_size,
        num_workers=args.num_workers, drop_last=drop_last, task_collate_fn=task_collate_fn)

    def metrics_func(model, epoch, output_predictions=False):
        print_rank_0("calculating metrics by accuracy func in ORQA...")
        if args.task != "RET-FINETUNE-NQ":
            raise AssertionError(f"{args.task} Task not supported")
        t0 = time.time()
        stats, total = retrieval_loss(model, dataloader)
        print_rank_0(f"epoch:{epoch}" + "".join(f"|{k} = {v / total:.2f}"
                                                for k, v in stats.items()))
        print_rank_0(f"taken time to calcuate metrics {time.time() - t0:.3f}")
        return {k: float(v) / total for k, v in stats.items()}

    return metrics_func


@torch.no_grad()
def retrieval_loss(model, dataloader):
    """Per batch: scores = Q @ [C_pos ; C_neg]^T; label of question i is i.
    Accumulates sum of ranks and top-k hit counts (each DP-averaged)."""
    args = get_args()
    ks = list(args.retriever_report_topk_accuracies)
    stats = {"rank": 0.0, **{f"top{k}_acc": 0.0 for k in ks}}
    total = 0
    assert len(model) == 1
    m = model[0]
    m.eval()
    for batch in dataloader:
        (q, qm, qt, _, c, cm, ct, _, nc, ncm, nct, _ref) = process_batch(batch)
        if nc is not None:
            c, cm, ct = torch.cat([c, nc]), torch.cat([cm, ncm]), torch.cat([ct, nct])
        ql, cl = m(q, qm, qt, c, cm, ct)
        scores = ql.float() @ cl.float().t()
        if args.retriever_score_scaling:
            scores = scores / math.sqrt(args.hidden_size)
        n = ql.shape[0]
        labels = torch.arange(n, device=scores.device)
        order = torch.argsort(torch.softmax(scores, 1), dim=1, descending=True)
        pos = (order == labels[:, None]).float().argmax(1)  # 0-based rank of the positive
        vals = [pos.sum()] + [(pos < k).float().sum() for k in ks]
        red = average_losses_across_data_parallel_group(vals)
        stats["rank"] += float(red[0])
        for k, v in zip(ks, red[1:]):
            stats[f"top{k}_acc"] += float(v) * 100
        total += n
    m.train()
    return stats, total

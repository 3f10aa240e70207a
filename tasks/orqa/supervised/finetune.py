"""RET-FINETUNE-NQ: supervised dual-encoder retriever finetuning (reference
``tasks/orqa/supervised/finetune.py``).

In-batch negatives over the whole DP world: query and context embeddings are
all-gathered (gradient flows back to the local slice only), scored as
``Q_all @ C_all^T`` and trained with cross-entropy whose target for question
i of rank r is its own positive passage.  With ``--train_with_neg`` each
rank's contexts are ``[positives ; hard negatives]`` (negatives padded to the
largest count over ranks so the gather is rectangular), so the positive of
question i on rank r sits at column ``r * local_contexts + i``.
"""
import math
from functools import partial

import torch
import torch.distributed as dist
import torch.nn.functional as F

from epfl_megatron_amd import get_args, get_timers, get_tokenizer, print_rank_0
from epfl_megatron_amd.models import ModelType
from epfl_megatron_amd.models.biencoder_model import biencoder_model_provider
from epfl_megatron_amd.parallel import state
from epfl_megatron_amd.utils.misc import average_losses_across_data_parallel_group

from ... import finetune_utils
from .data import NQSupervisedDataset
from .eval_utils import accuracy_func_provider, process_batch, task_collate_fn


def get_group_world_size_rank():
    if not dist.is_initialized():
        return None, 0, 1
    g = state.get_data_parallel_group()
    return g, dist.get_rank(group=g), dist.get_world_size(group=g)


class _GatherDP(torch.autograd.Function):
    """All-gather along dim 0 over DP; backward keeps the local rows' gradient."""

    @staticmethod
    def forward(ctx, x):
        g, r, w = get_group_world_size_rank()
        ctx.rank, ctx.n = r, x.shape[0]
        if w == 1:
            return x
        parts = [torch.empty_like(x) for _ in range(w)]
        dist.all_gather(parts, x.contiguous(), group=g)
        return torch.cat(parts)

    @staticmethod
    def backward(ctx, grad):
        return grad[ctx.rank * ctx.n:(ctx.rank + 1) * ctx.n]


def check_and_append_tensor_for_gather(group, rank, world_size, input_):
    """Zero-pad dim 0 to the largest size over the DP group."""
    if world_size == 1:
        return input_
    n = torch.tensor([input_.shape[0]], device=input_.device)
    sizes = [torch.empty_like(n) for _ in range(world_size)]
    dist.all_gather(sizes, n, group=group)
    mx = int(torch.stack(sizes).max())
    if mx > input_.shape[0]:
        pad = [0] * (2 * input_.dim() - 1) + [mx - input_.shape[0]]
        input_ = F.pad(input_, pad)
    return input_


def cross_entropy_loss_func(local_queries, local_contexts, output_tensor):
    args = get_args()
    _, _, world = get_group_world_size_rank()
    ql, cl = output_tensor
    all_q, all_c = _GatherDP.apply(ql), _GatherDP.apply(cl)
    scores = all_q @ all_c.t()
    if args.retriever_score_scaling:
        scores = scores / math.sqrt(args.hidden_size)
    if args.train_with_neg:
        labels = torch.cat([torch.arange(r * local_contexts, r * local_contexts + local_queries)
                            for r in range(world)])
    else:
        labels = torch.arange(world * local_queries)
    labels = labels.to(scores.device)
    logp = F.log_softmax(scores.float(), dim=1)
    loss = F.nll_loss(logp, labels)
    correct = (logp.argmax(1) == labels).sum().float()
    red = average_losses_across_data_parallel_group([loss, correct])
    # gradient of the gathered loss reaches each rank only through its slice;
    # DP averaging divides by world, so scale back up (reference behaviour)
    return loss * state.get_data_parallel_world_size(), \
        {"lm loss": red[0], "correct_prediction_count": red[1]}


def orqa(Dataset):
    def forward_step(batch, model):
        timers = get_timers()
        timers("batch generator", log_level=2).start()
        b = finetune_utils._next_batch(batch)
        g, r, w = get_group_world_size_rank()
        (q, qm, qt, _, c, cm, ct, _, nc, ncm, nct, _ref) = process_batch(b)
        timers("batch generator").stop()
        if nc is not None:
            nc = check_and_append_tensor_for_gather(g, r, w, nc)
            ncm = check_and_append_tensor_for_gather(g, r, w, ncm)
            nct = check_and_append_tensor_for_gather(g, r, w, nct)
            c, cm, ct = torch.cat([c, nc]), torch.cat([cm, ncm]), torch.cat([ct, nct])
        out = model(q, qm, qt, c, cm, ct)
        return out, partial(cross_entropy_loss_func, q.shape[0], c.shape[0])

    def train_valid_datasets_provider():
        args, tok = get_args(), get_tokenizer()
        return (Dataset("training", args.train_data, tok, args.retriever_seq_length,
                        evaluate=False),
                Dataset("validation", args.valid_data, tok, args.retriever_seq_length,
                        evaluate=True))

    def model_provider(pre_process=True, post_process=True):
        args = get_args()
        print_rank_0(f"building retriever model for {args.task} ...")
        return biencoder_model_provider(
            only_context_model=False, only_query_model=False,
            biencoder_shared_query_context_model=args.biencoder_shared_query_context_model,
            pre_process=pre_process, post_process=post_process,
            model_type=ModelType.encoder_or_decoder)

    def single_dataset_provider(datapath):
        args = get_args()
        name = datapath[0].split("/")[-1].split(".")[0]
        return Dataset(name, datapath, get_tokenizer(), args.retriever_seq_length, evaluate=True)

    return finetune_utils.finetune(
        train_valid_datasets_provider, model_provider, ModelType.encoder_or_decoder,
        forward_step=forward_step,
        end_of_epoch_callback_provider=lambda: accuracy_func_provider(single_dataset_provider),
        task_collate_fn=task_collate_fn)


def main():
    args = get_args()
    if args.task != "RET-FINETUNE-NQ":
        raise NotImplementedError(f"ORQA task {args.task} is not implemented.")
    return orqa(NQSupervisedDataset)

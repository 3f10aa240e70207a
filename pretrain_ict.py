"""Pretrain a BERT bi-encoder with the Inverse Cloze Task — reference
``pretrain_ict.py``.  In-batch negatives over the whole data-parallel batch:
query/context embeddings are all-gathered across DP before the score matrix."""
import math
from functools import partial

import torch
import torch.distributed as dist
import torch.nn.functional as F

from epfl_megatron_amd import get_args, get_timers, print_rank_0
from epfl_megatron_amd.data.dataset_utils import build_train_valid_test_datasets
from epfl_megatron_amd.data.realm_dataset_utils import get_ict_batch
from epfl_megatron_amd.initialize import initialize_megatron
from epfl_megatron_amd.models import ModelType, biencoder_model_provider
from epfl_megatron_amd.parallel import state as mpu
from epfl_megatron_amd.training import pretrain
from epfl_megatron_amd.utils.misc import average_losses_across_data_parallel_group


def pretrain_ict_model_provider(pre_process=True, post_process=True):
    args = get_args()
    return biencoder_model_provider(
        only_context_model=False, only_query_model=False,
        biencoder_shared_query_context_model=args.biencoder_shared_query_context_model,
        pre_process=pre_process, post_process=post_process,
        model_type=ModelType.encoder_or_decoder)


class AllgatherFromDataParallelRegion(torch.autograd.Function):
    """[b, d] -> [dp * b, d] across the data-parallel group; backward keeps
    this rank's slice."""

    @staticmethod
    def forward(ctx, x):
        if x.dim() != 2:
            raise AssertionError("expected [b, d]")
        group = mpu.get_data_parallel_group()
        world = dist.get_world_size(group=group)
        parts = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(parts, x.contiguous(), group=group)
        parts[dist.get_rank(group=group)] = x
        return torch.cat(parts, dim=0).contiguous()

    @staticmethod
    def backward(ctx, grad):
        group = mpu.get_data_parallel_group()
        world = dist.get_world_size(group=group)
        rank = dist.get_rank(group=group)
        return torch.split(grad, grad.shape[0] // world, dim=0)[rank].contiguous()


def loss_func(output_tensor):
    args = get_args()
    q, c = output_tensor
    if mpu.get_tensor_model_parallel_world_size() != 1:
        raise AssertionError("Model parallel size > 1 not supported for ICT")
    all_q = AllgatherFromDataParallelRegion.apply(q)
    all_c = AllgatherFromDataParallelRegion.apply(c)
    n = all_q.shape[0]
    scores = torch.matmul(all_q, all_c.t())
    if args.retriever_score_scaling:
        scores = scores / math.sqrt(args.hidden_size)
    logp = F.log_softmax(scores.float(), dim=1)
    order = torch.topk(logp, k=logp.shape[1], sorted=True).indices
    labels = torch.arange(n, device=logp.device)

    def topk_accuracy(k):
        hit = (order[:, :k] == labels[:, None]).any(dim=1).float().mean()
        return hit.reshape(1)

    accs = [topk_accuracy(int(k)) for k in args.retriever_report_topk_accuracies]
    loss = F.nll_loss(logp, labels, reduction="mean")
    reduced = average_losses_across_data_parallel_group([loss, *accs])
    # every rank sees the full-DP score matrix: undo the DP averaging of grads
    loss = loss * mpu.get_data_parallel_world_size()
    stats = {"loss": reduced[0]}
    stats.update({f"top{k}_acc": v * 100 for k, v in
                  zip(args.retriever_report_topk_accuracies, reduced[1:])})
    return loss, stats


def forward_step(data_iterator, model):
    timers = get_timers()
    timers("batch-generator", log_level=2).start()
    q_tok, q_mask, c_tok, c_mask, _ = get_ict_batch(data_iterator)
    timers("batch-generator").stop()
    q_types = torch.zeros_like(q_tok)
    c_types = torch.zeros_like(c_tok)
    return model(q_tok, q_mask, q_types, c_tok, c_mask, c_types), partial(loss_func)


def train_valid_test_datasets_provider(train_val_test_num_samples):
    args = get_args()
    print_rank_0("> building train, validation, and test datasets for BERT ICT...")
    ds = build_train_valid_test_datasets(
        data_prefix=args.data_path, data_impl=args.data_impl, splits_string=args.split,
        train_valid_test_num_samples=train_val_test_num_samples, max_seq_length=args.seq_length,
        masked_lm_prob=args.mask_prob, short_seq_prob=args.short_seq_prob, seed=args.seed,
        skip_warmup=(not args.mmap_warmup), binary_head=False, dataset_type="ict")
    print_rank_0("> finished creating BERT ICT datasets ...")
    return ds


def main(args_list=None):
    initialize_megatron(None, {"tokenizer_type": "BertWordPieceLowerCase"}, args_list=args_list)
    return pretrain(get_args(), train_valid_test_datasets_provider,
                    pretrain_ict_model_provider, ModelType.encoder_or_decoder, forward_step)


if __name__ == "__main__":
    main()

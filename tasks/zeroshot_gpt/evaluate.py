"""Zero-shot LM evaluation: WikiText perplexity and LAMBADA accuracy
(reference tasks/zeroshot_gpt/evaluate.py).

Pipeline-aware forward-only loop over this DP rank's share of the samples
(rank r takes samples r, r + dp, ...); the per-rank totals are summed with
one all-reduce over the data-parallel group at the end, so ranks may hold
different numbers of batches (no padded duplicates).
"""
import math

import numpy as np

import torch
import torch.distributed as dist

from epfl_megatron_amd import get_args, get_tokenizer, print_rank_0
from epfl_megatron_amd.checkpointing import load_checkpoint
from epfl_megatron_amd.models import ModelType
from epfl_megatron_amd.parallel import state
from epfl_megatron_amd.parallel.pipeline.p2p import recv_forward, send_forward
from epfl_megatron_amd.training import get_model
from epfl_megatron_amd.utils.misc import get_ltor_masks_and_position_ids, unwrap_model
from .datasets import build_dataset


def _model_provider(eval_metric):
    def provider(pre_process=True, post_process=True):
        import finetune
        args = get_args()
        model = finetune.model_provider(pre_process, post_process)
        # accuracy needs full-vocab argmax; loss works on vocab-parallel logits
        model.parallel_output = eval_metric == "loss"
        return model
    return provider


def _device():
    return torch.device("cpu") if dist.get_backend() == "gloo" else \
        torch.device("cuda", torch.cuda.current_device())


def process_batch(batch):
    args = get_args()
    dev = _device()
    loss_mask = batch["pad_mask"].long().to(dev)
    toks = batch["text"].long().to(dev)
    labels, tokens = toks[:, 1:].contiguous(), toks[:, :-1].contiguous()
    attn, _, pos = get_ltor_masks_and_position_ids(tokens, get_tokenizer().eod,
                                                   args.reset_position_ids,
                                                   args.reset_attention_mask, args.eod_mask_loss)
    return tokens, labels, attn, pos, loss_mask


def forward_step(batch, model, eval_metric):
    tokens, labels, attn, pos, loss_mask = process_batch(batch)
    args = get_args()
    b, s = tokens.shape
    if args.sequence_parallel:
        s //= state.get_tensor_model_parallel_world_size()
    shape = (s, b, args.hidden_size)
    x = recv_forward(shape, dtype_=args.params_dtype)
    unwrap_model(model).set_input_tensor(x)
    pos_arg = pos if args.position_embedding_type.name == "absolute" else None
    if eval_metric == "loss":
        # per-token vocab-parallel CE computed inside the model: [b, s]
        out = model(tokens, pos_arg, attn, labels=labels)
    elif eval_metric == "accuracy":
        out = model(tokens, pos_arg, attn)  # gathered logits [b, s, v]
    else:
        raise NotImplementedError(eval_metric)
    send_forward(out, shape, dtype_=args.params_dtype)
    if not state.is_pipeline_last_stage():
        return None
    if eval_metric == "loss":
        return (out.float() * loss_mask.float()).sum()
    correct = (out.argmax(-1) == labels) | (loss_mask == 0)
    return correct.all(-1).float().sum()


def evaluate(dataset, model, eval_metric):
    args = get_args()
    model.eval()
    dp, r = state.get_data_parallel_world_size(), state.get_data_parallel_rank()
    idx = list(range(r, len(dataset), dp))
    mbs = args.micro_batch_size
    total = torch.zeros(1, dtype=torch.float64, device=_device())
    with torch.no_grad():
        for it, start in enumerate(range(0, len(idx), mbs)):
            if it % args.log_interval == 0:
                print_rank_0(f"> working on iteration: {it}")
            items = [dataset[i] for i in idx[start:start + mbs]]
            batch = {k: torch.as_tensor(np.stack([d[k] for d in items]))
                     for k in items[0]}
            out = forward_step(batch, model, eval_metric)
            if out is not None:
                total += out.double()
    if state.is_pipeline_last_stage():
        dist.all_reduce(total, group=state.get_data_parallel_group())
    return total.item()


def evaluate_and_print_results(task, dataset, model, eval_metric):
    out = evaluate(dataset, model, eval_metric)
    res = {}
    if state.is_pipeline_last_stage() and state.get_tensor_model_parallel_rank() == 0:
        line = f" validation results on {task} | "
        if eval_metric == "loss":
            val_loss = out / (dataset.num_tokenized_tokens - 1)
            ratio = (dataset.num_tokenized_tokens - 1) / (dataset.num_original_tokens - 1)
            res = dict(loss=val_loss, ppl=math.exp(min(20, val_loss)),
                       adjusted_ppl=math.exp(min(20, val_loss * ratio)), token_ratio=ratio)
            line += (f"avg loss: {val_loss:.4E} | ppl: {res['ppl']:.4E} | adjusted ppl: "
                     f"{res['adjusted_ppl']:.4E} | token ratio: {ratio} |")
        else:
            acc = out / len(dataset)
            res = dict(correct=out, total=len(dataset), accuracy=acc)
            line += (f"number correct: {out:.4E} | total examples: {len(dataset):.4E} | "
                     f"avg accuracy: {acc:.4E}")
        print("-" * (len(line) + 1))
        print(line)
        print("-" * (len(line) + 1), flush=True)
    return res


def main():
    args = get_args()
    if args.num_layers_per_virtual_pipeline_stage is not None:
        raise SystemExit("Interleaved pipeline schedule is not supported for evaluation.")
    metric = {"LAMBADA": "accuracy", "WIKITEXT103": "loss"}.get(args.task)
    if metric is None:
        raise NotImplementedError(f"{args.task} task is not implemented.")
    model = get_model(_model_provider(metric), ModelType.encoder_or_decoder, wrap_with_ddp=False)
    if args.load is not None:
        load_checkpoint(model, None, None)
    res = evaluate_and_print_results(args.task, build_dataset(args.task), model[0], metric)
    print_rank_0("done :-)")
    return res

"""Run this framework's model and a Hugging Face reference side by side
(reference ``verify_correctness.py``).

    python verify_correctness.py --model_name llama2 --load MEGATRON_CKPT \
        --huggingface_cache HF_DIR [--huggingface_device cuda:1] \
        --data_path CORPUS | --synthetic_data  [model / tokenizer flags]

For 10 iterations of real (or synthetic) batches it prints the max / mean
absolute logit error and the loss error between the two models.  The
baseline is a local Hugging Face directory (``LlamaForCausalLM`` /
``FalconForCausalLM``; no downloads).  ``--load`` may also be a Hugging Face
directory, in which case that converted model is compared instead (the
reference's ``hf_our_provider``).  Model-shape flags are taken from the
checkpoint (``--use_checkpoint_args`` is on by default).
"""
from pathlib import Path

import torch

from epfl_megatron_amd import get_args
from epfl_megatron_amd.config.arguments import parse_args
from epfl_megatron_amd.initialize import initialize_megatron
from epfl_megatron_amd.training import (_setup_model_and_optimizer,
                                        build_train_valid_test_data_iterators)

from finetune import extra_args, get_batch, loss_func, model_provider, \
    train_valid_test_datasets_provider


def is_megatron_path(path):
    return path is not None and (Path(path) / "latest_checkpointed_iteration.txt").exists()


def hf_provider(name, path, device):
    import transformers
    cls = transformers.FalconForCausalLM if name == "falcon" else transformers.LlamaForCausalLM
    model = cls.from_pretrained(str(path), torch_dtype=torch.float32)
    return model.eval().requires_grad_(False).to(device)


def hf_forward(model, batch):
    device = next(model.parameters()).device
    tokens, labels, loss_mask, attention_mask, position_ids = [t.to(device) for t in batch]
    out = model(input_ids=tokens, labels=tokens)
    # HF shifts labels internally; compare the loss over the same positions
    logits = out["logits"].float()
    logp = torch.log_softmax(logits, dim=-1)
    nll = -logp.gather(-1, labels.unsqueeze(-1)).squeeze(-1)
    loss = (nll * loss_mask).sum() / loss_mask.sum()
    return logits, loss


def mega_provider():
    args = get_args()
    from epfl_megatron_amd.models import ModelType
    model, _, _ = _setup_model_and_optimizer(model_provider, ModelType.encoder_or_decoder,
                                             args=args)
    if len(model) != 1:
        raise AssertionError("correctness verification only supports unsharded models")
    from epfl_megatron_amd.utils.misc import unwrap_model
    return unwrap_model(model)[0].eval().requires_grad_(False)


def mega_forward(model, batch):
    tokens, labels, loss_mask, attention_mask, position_ids = batch
    pos = position_ids if get_args().position_embedding_type.name == "absolute" else None
    with torch.no_grad():
        logits = model(tokens, pos, attention_mask, labels=None)
        losses = model(tokens, pos, attention_mask, labels=labels)
    loss, _ = loss_func(loss_mask, losses)
    if get_args().tensor_model_parallel_size > 1:
        raise AssertionError("run verification on a TP=1 checkpoint (re-shard first)")
    return logits.float(), loss


def verify_step(our_forward, our_model, base_forward, base_model, batch):
    our_logits, our_loss = our_forward(our_model, batch)
    base_logits, base_loss = base_forward(base_model, batch)
    v = min(our_logits.size(-1), base_logits.size(-1))  # padded vocab on our side
    our_logits, base_logits = our_logits[..., :v].cpu(), base_logits[..., :v].cpu()
    if our_logits.shape != base_logits.shape:
        raise AssertionError(f"ours={tuple(our_logits.shape)}, true={tuple(base_logits.shape)}")
    err = (our_logits - base_logits).abs()
    loss_err = (our_loss.float().cpu() - base_loss.float().cpu()).abs()
    print(f"Max absolute error in the logits: max={err.max():.6f}, avg={err.mean():.6f}")
    print(f"Abs loss error: {loss_err:.6f} Our loss: {our_loss.item():.3f}, "
          f"theirs: {base_loss.item():.3f}", flush=True)
    return err.max().item(), loss_err.item()


def main(iters=10):
    args = get_args()
    print("Starting megatron vs huggingface verification")
    if is_megatron_path(args.load):
        our_model, our_forward = mega_provider(), mega_forward
    else:
        print(f"NOTE: {args.load} is not a megatron checkpoint, assuming a Hugging Face one")
        our_model = hf_provider(args.model_name, args.load, args.baseline_device)
        our_forward = hf_forward
        args.iteration = 0
    base_model = hf_provider(args.model_name, args.cache_dir, args.baseline_device)
    data_iterator, _, _ = build_train_valid_test_data_iterators(
        train_valid_test_datasets_provider, args)
    results = []
    for it in range(iters):
        print(f"Iteration {it}...")
        results.append(verify_step(our_forward, our_model, hf_forward, base_model,
                                   get_batch(data_iterator)))
    return results


def extra_extra_args(parser):
    parser = extra_args(parser)
    g = parser.add_argument_group(title="huggingface")
    g.add_argument("--huggingface_cache", type=Path, default=None, dest="cache_dir",
                   help="local Hugging Face model directory of the baseline")
    default_dev = "cuda:1" if torch.cuda.device_count() > 1 else \
        ("cuda:0" if torch.cuda.is_available() else "cpu")
    g.add_argument("--huggingface_device", default=default_dev, dest="baseline_device")
    g.add_argument("--model_size", type=int, default=7)
    return parser


def defaults_for(load):
    d = {"micro_batch_size": 1, "use_checkpoint_args": True, "train_iters": 10, "lr": 1.0,
         "no_load_optim": True, "no_load_rng": True, "finetune": True}
    if not is_megatron_path(load):
        d.update({"num_layers": 1, "hidden_size": 8, "num_attention_heads": 1,
                  "seq_length": 2048, "max_position_embeddings": 2048})
    return d


if __name__ == "__main__":
    pre = parse_args(extra_extra_args)
    initialize_megatron(extra_extra_args, args_defaults=defaults_for(pre.load))
    main()

"""Headline benchmark: Llama-2-7B bf16 training throughput on N MI355X (one node).

Metric (BASELINE.json): tokens/s (+ MFU) for Llama-2-7B bf16 with pure data
parallelism (weak scaling: each GPU processes a fixed per-GPU batch).  The
model is the real Llama-2-7B architecture (32 layers, h=4096, 32 heads,
ffn 11008, vocab 32000, RMSNorm, SwiGLU, RoPE, untied head) with random init;
data is synthetic tokens (no corpus/network).  Every timed step is a complete
training step through the framework: forward, backward, bucketed RCCL gradient
reduction (reduce-scatter with the distributed optimizer when N > 1), grad-norm
clipping, fused AdamW update, parameter all-gather.

``value`` is the whole-job aggregate tokens/s; ``vs_baseline`` compares the
per-GPU rate with the reference's published A100 figure (BASELINE.md P1':
~890 tokens/s/GPU for Llama-2-7B, seq 1024).

Usage (driver contract):
    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

REF_TOKENS_PER_SEC_PER_GPU = 890.0  # BASELINE.md P1' (8x A100, seq 1024)


def _parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seq_len", type=int, default=1024)
    ap.add_argument("--micro_batch", type=int, default=16)
    ap.add_argument("--num_micro", type=int, default=2, help="micro-batches per GPU per step")
    ap.add_argument("--model", default="llama2-7b", choices=["llama2-7b", "llama2-13b", "tiny"])
    ap.add_argument("--recompute", default=None, choices=[None, "selective", "full"])
    ap.add_argument("--no_dist_opt", action="store_true")
    ap.add_argument("--bucket_mb", type=float, default=512.0)
    return ap.parse_args(argv)


MODELS = {
    "llama2-7b": dict(num_layers=32, hidden_size=4096, num_attention_heads=32,
                      ffn_hidden_size=11008),
    "llama2-13b": dict(num_layers=40, hidden_size=5120, num_attention_heads=40,
                       ffn_hidden_size=13824),
    "tiny": dict(num_layers=2, hidden_size=256, num_attention_heads=4, ffn_hidden_size=688),
}


def main(argv=None):
    a = _parse(argv)
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus and not (world == 1 and a.gpus == 1):
        print(f"warning: WORLD_SIZE={world} but --gpus={a.gpus}", file=sys.stderr)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    on_gpu = torch.cuda.is_available()
    model = a.model if on_gpu else "tiny"
    shape = MODELS[model]
    dp = world
    gbs = a.micro_batch * a.num_micro * dp
    argv = [
        "--num_layers", str(shape["num_layers"]), "--hidden_size", str(shape["hidden_size"]),
        "--num_attention_heads", str(shape["num_attention_heads"]),
        "--ffn_hidden_size", str(shape["ffn_hidden_size"]),
        "--seq_length", str(a.seq_len), "--max_position_embeddings", str(max(4096, a.seq_len)),
        "--position_embedding_type", "rotary", "--use_rms_norm", "--glu_activation", "swiglu",
        "--no_tie_embed_logits", "--layernorm_epsilon", "1e-5", "--hidden_dropout", "0.0",
        "--attention_dropout", "0.0", "--no_bias_gelu_fusion", "--no_bias_dropout_fusion",
        "--use_flash_attn", "--micro_batch_size", str(a.micro_batch),
        "--global_batch_size", str(gbs), "--train_iters", str(a.steps + a.warmup + 1),
        "--lr", "3e-4", "--min_lr", "3e-5", "--lr_decay_style", "cosine", "--lr_warmup_iters", "1",
        "--adam_beta2", "0.95", "--adam_eps", "1e-5", "--weight_decay", "0.1",
        "--clip_grad", "1.0", "--log_interval", "1000000", "--eval_interval", "1000000",
        "--eval_iters", "0", "--tokenizer_type", "NullTokenizer", "--synthetic_data",
        "--synthetic_vocab_size", "32000", "--make_vocab_size_divisible_by", "128",
        "--num_workers", "0", "--ddp_bucket_size_mb", str(a.bucket_mb),
        "--model_name", "llama2",
    ]
    if on_gpu:
        argv += ["--bf16"]
    else:
        argv += ["--distributed_backend", "gloo"]
    if dp > 1 and not a.no_dist_opt:
        argv += ["--use_distributed_optimizer"]
    if a.recompute:
        argv += ["--recompute_granularity", a.recompute]
        if a.recompute == "full":
            argv += ["--recompute_method", "uniform", "--recompute_num_layers", "1"]

    import finetune
    from epfl_megatron_amd import get_args, get_timers
    from epfl_megatron_amd.initialize import initialize_megatron
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.training import (_setup_model_and_optimizer,
                                            build_train_valid_test_data_iterators, train_step)
    from epfl_megatron_amd.utils.flops import flops_per_token
    import torch.distributed as dist

    initialize_megatron(finetune.extra_args, {"tokenizer_type": "NullTokenizer"}, args_list=argv)
    args = get_args()
    chunks, optimizer, sched = _setup_model_and_optimizer(finetune.model_provider,
                                                         ModelType.encoder_or_decoder, args=args)
    train_it, _, _ = build_train_valid_test_data_iterators(
        finetune.train_valid_test_datasets_provider, args)
    for m in chunks:
        m.train()

    def sync():
        if on_gpu:
            torch.cuda.synchronize()
        dist.barrier()

    def step():
        out = train_step(finetune.forward_step, train_it, chunks, optimizer, sched, args)
        args.consumed_train_samples += gbs
        return out

    for _ in range(a.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    last = None
    for _ in range(a.steps):
        last = step()
    sync()
    dt = time.perf_counter() - t0
    # max over ranks
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    tokens = gbs * a.seq_len * a.steps
    tok_s = tokens / dt
    per_gpu = tok_s / world
    fpt = flops_per_token(args)
    mfu = per_gpu * fpt / (args.peak_tflops * 1e12)
    loss = None
    if last is not None and last[0]:
        loss = float(last[0]["lm loss"])
    if dist.get_rank() == 0:
        rec = {
            "metric": "Llama-2-7B bf16 training throughput, tokens/s aggregate over GPUs "
                      "(BASELINE metric: tokens/sec/GPU + MFU; per-GPU = value / n_gpus)",
            "value": round(tok_s, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * dt / a.steps, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(per_gpu / REF_TOKENS_PER_SEC_PER_GPU, 3),
            "dtype": "bf16" if on_gpu else "fp32",
            "data": "synthetic",
            "config": {"model": "Llama-2-7B" if model == "llama2-7b" else model,
                       "global_batch": gbs, "seq_len": a.seq_len,
                       "micro_batch": a.micro_batch,
                       "parallelism": f"dp{world}" + ("+distopt" if dp > 1 and not a.no_dist_opt
                                                      else "")},
            "tokens_per_sec_per_gpu": round(per_gpu, 1),
            "mfu": round(mfu, 4),
            "tflops_per_gpu": round(per_gpu * fpt / 1e12, 1),
            "flops_per_token": fpt,
            "peak_tflops_assumed": args.peak_tflops,
            "final_loss": loss,
            "max_mem_gb": (round(torch.cuda.max_memory_allocated() / 2**30, 1)
                           if on_gpu else None),
        }
        print(json.dumps(rec), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

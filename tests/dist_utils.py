"""Multi-process CPU/gloo harness (the reference had no CPU path).

``run_dist(fn, world_size, *args)`` spawns ``world_size`` processes, sets the
torchrun-style env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR=127.0.0.1), calls
``fn(rank, world_size, *args)`` in each and re-raises the first failure.
Results are returned through a multiprocessing queue (``fn`` return values).
"""
import io
import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, args, q, env=None):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), OMP_NUM_THREADS="1")
    if env:
        os.environ.update(env)
    import torch
    torch.set_num_threads(1)
    try:
        out = fn(rank, world, *args)
        # results travel as bytes, not as shared-memory tensors: a tensor put on
        # the queue is backed by a segment the exiting worker may already have
        # released when the parent unpickles it (FileNotFoundError)
        buf = io.BytesIO()
        torch.save(out, buf)
        q.put((rank, "ok", buf.getvalue()))
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, "err", traceback.format_exc()))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            try:
                dist.barrier()
                dist.destroy_process_group()
            except Exception:
                pass


def run_dist(fn, world_size, *args, timeout=600, env=None):
    """``env``: extra environment for the ranks, applied before the GPU is
    touched (e.g. ``HIP_VISIBLE_DEVICES=""`` for a CPU reference run)."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world_size, port, fn, args, q, env))
             for r in range(world_size)]
    for p in procs:
        p.start()
    results = {}
    errors = []
    for _ in range(world_size):
        rank, status, payload = q.get()
        if status == "ok":
            import torch
            # (bytes written by this harness's own worker above)
            results[rank] = torch.load(io.BytesIO(payload), weights_only=False)
        else:
            errors.append(f"rank {rank}:\n{payload}")
            break
    for p in procs:
        p.join(timeout=5 if errors else timeout)
        if p.is_alive():
            p.terminate()
    if errors:
        raise AssertionError("\n".join(errors))
    return [results[r] for r in range(world_size)]


def init_framework(argv, extra_args_provider=None):
    """initialize_megatron on the gloo backend with an explicit flag list."""
    from epfl_megatron_amd.initialize import initialize_megatron
    base = ["--distributed_backend", "gloo", "--num_workers", "0"]
    return initialize_megatron(extra_args_provider, {"tokenizer_type": "NullTokenizer"},
                               args_list=base + list(argv))


TINY_LLAMA = ["--num_layers", "2", "--hidden_size", "64", "--num_attention_heads", "4",
              "--ffn_hidden_size", "128", "--seq_length", "16", "--max_position_embeddings", "32",
              "--position_embedding_type", "rotary", "--use_rms_norm", "--glu_activation",
              "swiglu", "--no_tie_embed_logits", "--hidden_dropout", "0.0",
              "--attention_dropout", "0.0", "--no_bias_gelu_fusion", "--no_bias_dropout_fusion",
              "--tokenizer_type", "NullTokenizer", "--synthetic_vocab_size", "250",
              "--make_vocab_size_divisible_by", "8", "--use_cpu_initialization",
              "--model_name", "llama2", "--lr", "1e-3", "--min_lr", "1e-4",
              "--lr_decay_style", "cosine", "--train_iters", "4", "--seed", "1234",
              "--log_interval", "1000", "--eval_iters", "0", "--eval_interval", "1000",
              "--synthetic_data", "--clip_grad", "1.0", "--weight_decay", "0.1"]

TINY_GPT = ["--num_layers", "2", "--hidden_size", "64", "--num_attention_heads", "4",
            "--seq_length", "16", "--max_position_embeddings", "32",
            "--hidden_dropout", "0.0", "--attention_dropout", "0.0",
            "--tokenizer_type", "NullTokenizer", "--synthetic_vocab_size", "250",
            "--make_vocab_size_divisible_by", "8", "--use_cpu_initialization",
            "--model_name", "gpt", "--lr", "1e-3", "--train_iters", "4", "--seed", "1234",
            "--log_interval", "1000", "--eval_iters", "0", "--eval_interval", "1000",
            "--synthetic_data", "--use_bias"]

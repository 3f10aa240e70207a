"""Serving benchmark: KV-cached greedy generation throughput on 1 GPU.

Llama-2-7B architecture, random init, bf16.  For each batch size: prefill a
128-token prompt, then decode 128 tokens one step at a time (greedy argmax on
the device, no host sync inside the loop); reports prefill ms and decode
tokens/s (batch x steps / decode time).  The decode step runs the framework's
inference path: fused QKV GEMM, RoPE pass with the position offset, KV-cache
write, split-key decode attention (csrc/flash_decode.hip), SwiGLU, RMSNorm.

Usage: python scripts/serve_bench.py [--batches 1,8,32] [--model llama2-7b]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,8,32")
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--gen", type=int, default=128)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--graph", action="store_true",
                    help="decode steps replayed from one captured hipGraph (inference/hip_graph.py)")
    a = ap.parse_args()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29561"),
                      RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import torch
    import finetune
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.initialize import initialize_megatron
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.training import get_model
    from epfl_megatron_amd.inference.forward_step import InferenceParams
    from epfl_megatron_amd.inference.hip_graph import GraphedGreedyDecoder

    argv = ["--num_layers", str(a.layers), "--hidden_size", "4096", "--num_attention_heads", "32",
            "--ffn_hidden_size", "11008", "--seq_length", "4096", "--max_position_embeddings",
            "4096", "--position_embedding_type", "rotary", "--use_rms_norm", "--glu_activation",
            "swiglu", "--no_tie_embed_logits", "--model_name", "llama2", "--use_flash_attn",
            "--hidden_dropout", "0.0", "--attention_dropout", "0.0", "--bf16",
            "--tokenizer_type", "NullTokenizer", "--synthetic_vocab_size", "32000",
            "--make_vocab_size_divisible_by", "128", "--micro_batch_size", "1",
            "--global_batch_size", "1", "--train_iters", "1", "--lr", "1e-4"]
    initialize_megatron(finetune.extra_args, {"tokenizer_type": "NullTokenizer"}, args_list=argv)
    model = get_model(finetune.model_provider, ModelType.encoder_or_decoder, wrap_with_ddp=False)
    m = model[0].eval()
    res = []
    for B in [int(x) for x in a.batches.split(",")]:
        total = a.prompt + a.gen
        torch.manual_seed(0)
        prompt = torch.randint(0, 32000, (B, a.prompt), device="cuda")
        pos = torch.arange(total, device="cuda")[None].expand(B, -1)
        with torch.no_grad():
            ip = InferenceParams(B, total)
            for rep in range(2):  # rep 0 warms up allocator / kernels
                if not a.graph:
                    ip = InferenceParams(B, total)
                ip.sequence_len_offset = 0  # graph mode: same caches, prefill again
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                logits = m(prompt, pos[:, :a.prompt], None, inference_params=ip)
                nxt = logits[:, -1].argmax(-1, keepdim=True)
                ip.sequence_len_offset += a.prompt
                if a.graph:  # capture (rep 0) / re-prime, outside the timed region
                    if rep == 0:
                        dec = GraphedGreedyDecoder(m, ip, B, a.gen)
                    dec.start(nxt, a.prompt)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                if a.graph:
                    for _ in range(a.prompt, total - 1):
                        dec.step()
                else:
                    for t in range(a.prompt, total - 1):
                        logits = m(nxt, pos[:, t:t + 1], None, inference_params=ip)
                        nxt = logits[:, -1].argmax(-1, keepdim=True)
                        ip.sequence_len_offset += 1
                torch.cuda.synchronize()
                t2 = time.perf_counter()
        steps = a.gen - 1
        r = {"batch": B, "graph": bool(a.graph), "prompt": a.prompt, "gen": a.gen, "prefill_ms": round(1e3 * (t1 - t0), 2),
             "decode_ms_per_step": round(1e3 * (t2 - t1) / steps, 3),
             "decode_tokens_per_s": round(B * steps / (t2 - t1), 1)}
        print(json.dumps(r), flush=True)
        res.append(r)
    return res


if __name__ == "__main__":
    main()

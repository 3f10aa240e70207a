"""Context-parallel attention cost per rank on one GPU (kernel side only, no
transfers): the W ranks of a zig-zag ring simulated one after another
(parallel/context.py ring_attention_simulated), forward + backward, against
one-GPU FlashAttention over the whole sequence.  Llama-2-7B heads.

    python scripts/cp_pair_bench.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    from epfl_megatron_amd.ops.attention import flash_attn_func
    from epfl_megatron_amd.parallel.context import ring_attention_simulated, zigzag_slice
    b, nq, hd = 1, 32, 128
    for s in (16384, 32768):
        q = torch.randn(b, s, nq, hd, device="cuda", dtype=torch.bfloat16)
        k, v, go = torch.randn_like(q), torch.randn_like(q), torch.randn_like(q)
        flops = 4 * b * nq * hd * s * s / 2 * 3.5  # causal fwd (2 GEMMs) + bwd (5 GEMMs)

        def full():
            qq, kk, vv = (t.detach().requires_grad_() for t in (q, k, v))
            flash_attn_func(qq, kk, vv, causal=True).backward(go)

        tf = timed(full)
        rec = {"s": s, "one_gpu_ms": round(tf * 1e3, 2), "one_gpu_tflops": round(flops / tf / 1e12, 1)}
        for W in (2, 4, 8):
            ch = lambda t: [zigzag_slice(t, 1, i, W).contiguous() for i in range(W)]  # noqa: E731
            qs, ks, vs, gs = ch(q), ch(k), ch(v), ch(go)
            tw = timed(lambda: ring_attention_simulated(qs, ks, vs, True, grad_outs=gs, zigzag=True),
                       reps=2)
            rec[f"cp{W}_per_rank_ms"] = round(tw / W * 1e3, 2)
            rec[f"cp{W}_tflops_per_rank"] = round(flops / W / (tw / W) / 1e12, 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

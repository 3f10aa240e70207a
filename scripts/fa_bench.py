"""FlashAttention fwd/bwd timing (1 GPU), causal, bf16.

    python scripts/fa_bench.py [b,s,nq,nkv,hd ...]

Default shapes: the Llama-2-7B training shape (8 x 1024, 32 heads) and the
seq-4096 one.  Per shape: median over 20 timed forward calls and over 10
forward+backward pairs (backward time = pair - forward).  EMA_FA_WAVES=4|8
forces the forward / dQ grid form.
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops.attention import flash_attn_func  # noqa: E402


def run(b, s, nq, nkv, hd):
    torch.manual_seed(0)
    q = torch.randn(b, s, nq, hd, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(b, s, nkv, hd, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(b, s, nkv, hd, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(b, s, nq, hd, device="cuda", dtype=torch.bfloat16)
    fl = 4.0 * b * nq * s * s * hd / 2  # causal
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    tf = []
    with torch.no_grad():
        for it in range(23):
            e0, e1 = ev(), ev()
            e0.record()
            flash_attn_func(q, k, v, causal=True)
            e1.record()
            torch.cuda.synchronize()
            if it >= 3:
                tf.append(e0.elapsed_time(e1))
    tb = []
    for it in range(12):
        e0, e1, e2 = ev(), ev(), ev()
        e0.record()
        o = flash_attn_func(q, k, v, causal=True)
        e1.record()
        o.backward(do)
        e2.record()
        torch.cuda.synchronize()
        if it >= 2:
            tb.append(e1.elapsed_time(e2))
        q.grad = k.grad = v.grad = None
    f, bw = statistics.median(tf), statistics.median(tb)
    print(f"b={b} s={s} nq={nq} nkv={nkv} hd={hd}: fwd {f * 1e3:.1f} us ({fl / f / 1e9:.0f} TF/s)  "
          f"bwd {bw * 1e3:.1f} us ({2.5 * fl / bw / 1e9:.0f} TF/s)", flush=True)


def main():
    shapes = sys.argv[1:] or ["8,1024,32,32,128", "2,4096,32,32,128"]
    for sh in shapes:
        run(*[int(v) for v in sh.split(",")])


if __name__ == "__main__":
    main()

"""FlashAttention fwd/bwd timing at the Llama-2-7B training shape (1 GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops.attention import flash_attn_func  # noqa: E402


def main():
    b, s, nq, nkv, hd = 8, 1024, 32, 32, 128
    if len(sys.argv) > 1:
        b, s, nq, nkv, hd = [int(v) for v in sys.argv[1].split(",")]
    torch.manual_seed(0)
    q = torch.randn(b, s, nq, hd, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(b, s, nkv, hd, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(b, s, nkv, hd, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(b, s, nq, hd, device="cuda", dtype=torch.bfloat16)
    fl = 4.0 * b * nq * s * s * hd / 2  # causal
    for it in range(4):
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        o = flash_attn_func(q, k, v, causal=True)
        e[1].record()
        o.backward(do)
        e[2].record()
        torch.cuda.synchronize()
        tf, tb = e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2])
        print(f"iter {it}: fwd {tf * 1e3:.1f} us ({fl / tf / 1e9:.0f} TF/s)  "
              f"bwd {tb * 1e3:.1f} us ({2.5 * fl / tb / 1e9:.0f} TF/s)", flush=True)
        q.grad = k.grad = v.grad = None


if __name__ == "__main__":
    main()

"""Decode attention keys-per-wave A/B (csrc/flash_decode.hip): the same
single-token attention at KPW = 64 / 16 / 8 keys per wave (chunk = 4 KPW keys
per workgroup, in-kernel combine when a sequence spans several chunks) and the
automatic pick.  Event-timed loops of back-to-back launches; run it under
``rocprofv3 --kernel-trace --stats`` for per-kernel times (the kernel name
carries KPW).  Usage: python scripts/decode_kpw_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402
from epfl_megatron_amd.ops.attention import attention_ref, _bsnd_strides  # noqa: E402


def run(b, cap, n, nq, nkv, hd, kpw, reps=50):
    """cap = cache capacity (the launch's sk), n = valid keys (device kv_len)."""
    torch.manual_seed(0)
    kmem = torch.randn(cap, b, nkv, hd, device="cuda", dtype=torch.bfloat16)
    vmem = torch.randn(cap, b, nkv, hd, device="cuda", dtype=torch.bfloat16)
    q = torch.randn(b, 1, nq, hd, device="cuda", dtype=torch.bfloat16)
    k, v = kmem.transpose(0, 1), vmem.transpose(0, 1)
    kv_len = torch.tensor([n], device="cuda", dtype=torch.int32)
    out = torch.empty(b, 1, nq, hd, device="cuda", dtype=torch.bfloat16)
    r = nq // nkv
    scale = hd ** -0.5

    def call():
        ext().flash_decode(q, k, v, out, b, cap, nq, nkv, hd, list(_bsnd_strides(q, r)),
                           list(_bsnd_strides(k, 1)[:3]), list(_bsnd_strides(v, 1)[:3]),
                           [out.stride(0), out.stride(1), out.stride(2)], float(scale), kv_len, kpw)

    call()
    torch.cuda.synchronize()
    ref = attention_ref(q.float(), k[:, :n].float(), v[:, :n].float(), False, scale)
    err = (out.float() - ref).abs().max().item()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3, err


if __name__ == "__main__":
    for sh in ((1, 256, 192, 32, 32, 128), (8, 256, 192, 32, 32, 128), (1, 2048, 1500, 32, 32, 128),
               (1, 4096, 3000, 64, 8, 128), (16, 4096, 3000, 64, 8, 128), (4, 2048, 1000, 71, 1, 64)):
        row = []
        for kpw in (0, 64, 16, 8):
            us, err = run(*sh, kpw)
            assert err < 3e-2, (sh, kpw, err)
            row.append(f"{'auto' if kpw == 0 else kpw}: {us:6.1f} us")
        print(f"b={sh[0]} cap={sh[1]} kv_len={sh[2]} nq={sh[3]} nkv={sh[4]} hd={sh[5]}  " + "  ".join(row),
              flush=True)

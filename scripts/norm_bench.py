"""RMSNorm fwd/bwd timing at the Llama-2-7B training shape (rows = mbs*seq, H = 4096)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402


def main():
    rows, H = 16384, 4096
    x = torch.randn(rows, H, device="cuda", dtype=torch.bfloat16)
    r = torch.randn_like(x)
    dy = torch.randn_like(x)
    w = torch.ones(H, device="cuda", dtype=torch.bfloat16)
    y, rstd, s = ext().rmsnorm_fwd(x, w, 1e-5, r)
    mb = rows * H * 2 / 1e6
    for name, fn, nbytes in [
        ("fwd+res", lambda: ext().rmsnorm_fwd(x, w, 1e-5, r), 4 * mb),
        ("bwd", lambda: ext().rmsnorm_bwd(dy, s, w, rstd), 3 * mb),
        ("bwd+dres", lambda: ext().rmsnorm_bwd(dy, s, w, rstd, r), 4 * mb),
    ]:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"{name}: {us:.1f} us  ({nbytes / us:.2f} TB/s of essential traffic)", flush=True)


if __name__ == "__main__":
    main()

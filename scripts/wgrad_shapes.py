"""wgrad kernel TF/s over a set of (N, K) shapes at M = 16384 (isolated)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402
from wgrad_bench import _time  # noqa: E402

M = 16384
for spec in sys.argv[1:]:
    N, K = (int(v) for v in spec.split("x"))
    dY = torch.rand(M, N, device="cuda", dtype=torch.bfloat16) - 0.5
    X = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) - 0.5
    G = torch.zeros(N, K, device="cuda", dtype=torch.float32)
    t = _time(lambda: ext().wgrad_gemm(dY, X, G, True))
    print(f"N={N} K={K} tiles={(N // 256) * (K // 256)}: {2.0 * M * N * K / t / 1e12:.1f} TF/s", flush=True)
    del dY, X, G

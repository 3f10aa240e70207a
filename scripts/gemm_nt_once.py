"""Profiling driver: one NT GEMM shape through hipBLASLt and both hand-written
variants (5 calls each), uniform-random bf16 operands.

    python scripts/gemm_nt_once.py [M N K]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402

M, N, K = [int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (16384, 4096, 11008))]
C = ext()
a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    torch.matmul(a, b.t(), out=out)
for v in (8, 4):
    C.gemm_nt_set_variant(v)
    for _ in range(5):
        C.gemm_nt(a, b, out)
torch.cuda.synchronize()
print("done", flush=True)

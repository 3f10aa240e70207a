"""Profiling driver for scripts/gemm_ablation.py: one shape, 3 calls each of the
persistent NT GEMM (modes 0 / 1 / 2) and hipBLASLt.  python scripts/gemm_ablation_once.py M N K"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402

M, N, K = [int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (16384, 4096, 11008))]
C = ext()
a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    torch.matmul(a, b.t(), out=c)
for mode in (0, 1, 2):
    for _ in range(3):
        C.gemm_nt_ablation(a, b, c, mode)
torch.cuda.synchronize()
print("done", flush=True)

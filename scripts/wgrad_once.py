"""Run the custom wgrad kernel on one Llama-7B shape a few times (profiling driver).

    python scripts/wgrad_once.py [N K [MODE]]   (MODE: 0 full, 1 no epilogue, 2 no loads)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402

N, K = [int(v) for v in (sys.argv[1:3] if len(sys.argv) > 2 else (22016, 4096))]
MODE = int(sys.argv[3]) if len(sys.argv) > 3 else 0
M = 16384
dY = torch.rand(M, N, device="cuda", dtype=torch.bfloat16) - 0.5
X = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) - 0.5
G = torch.zeros(N, K, device="cuda", dtype=torch.float32)
for _ in range(5):
    ext().wgrad_gemm_ablation(dY, X, G, MODE)
torch.cuda.synchronize()
print("done", flush=True)

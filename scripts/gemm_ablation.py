"""Where the persistent NT GEMM (csrc/gemm_nt.hip variant 6) loses time:
interleaved timing (one process, CDNA guide rule 24) of the full kernel, the
kernel without its K-loop DMA, the kernel with neither DMA nor fragment reads
(MFMA + barriers + epilogue), and hipBLASLt, on uniform-random bf16 operands.

    python scripts/gemm_ablation.py [M N K ...]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402


def _t(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    C = ext()
    args = [int(v) for v in sys.argv[1:]]
    shapes = [tuple(args[i:i + 3]) for i in range(0, len(args), 3)] or \
        [(16384, 4096, 4096), (16384, 4096, 11008), (16384, 11008, 4096)]
    for M, N, K in shapes:
        a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        modes = ((0, "production"), (1, "no_dma"), (2, "mfma_only"), (14, "burst(r4e)"))
        r = {k: [] for _, k in modes}
        r["hipblaslt"] = []
        for _ in range(5):
            for mode, k in modes:
                r[k].append(fl / _t(lambda: C.gemm_nt_ablation(a, b, c, mode)) / 1e12)
            r["hipblaslt"].append(fl / _t(lambda: torch.matmul(a, b.t(), out=c)) / 1e12)
        print(f"M={M} N={N} K={K}: " + "  ".join(
            f"{k} {statistics.median(v):7.1f}" for k, v in r.items()) + " TF/s", flush=True)


if __name__ == "__main__":
    main()

"""hipBLASLt heuristic pick (what torch.matmul runs) vs the best of the
top-N solutions (``_C.lt_algos`` + ``_C.lt_gemm``) on the plain NT products of
the Llama-2-7B step that stay on the library: forward X W^T and dgrad
dY (W^T)^T with the per-step cached W^T (M = 16384 tokens).

    python scripts/lt_retune.py [N_ALGOS]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402

M = 16384
SHAPES = {  # name: (N, K) of C[M, N] = A[M, K] B[N, K]^T
    "qkv.fwd": (12288, 4096), "dense.fwd": (4096, 4096), "fc2.fwd": (4096, 11008),
    "lm_head.fwd": (32000, 4096), "qkv.dgrad": (4096, 12288), "dense.dgrad": (4096, 4096),
    "fc1.dgrad": (4096, 22016), "lm_head.dgrad": (4096, 32000),
}


def _time(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    C = ext()
    n_algos = int(sys.argv[1]) if len(sys.argv) > 1 else 150
    torch.manual_seed(0)
    for name, (N, K) in SHAPES.items():
        A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        B = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        D = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        t_torch = min(_time(lambda: torch.matmul(A, B.t(), out=D), 8) for _ in range(2))
        algos = C.lt_algos(A, False, B, True, D, 0.0, 16)[:n_algos]
        best = (t_torch, None, "torch")
        for a in algos:
            fn = lambda: C.lt_gemm(A, False, B, True, D, 1.0, 0.0, a)  # noqa: E731
            try:
                t1 = _time(fn, 1)
                if t1 > 1.5 * t_torch:
                    continue
                t = min(_time(fn, 6) for _ in range(2))
            except RuntimeError:
                continue
            if t < best[0]:
                best = (t, a, C.lt_algo_name(a)[:90])
        print(f"{name:14s} torch {fl / t_torch / 1e12:7.1f} TF/s   best {fl / best[0] / 1e12:7.1f} "
              f"(x{t_torch / best[0]:.3f}, {len(algos)} algos)  {best[2]}", flush=True)
        del A, B, D


if __name__ == "__main__":
    main()

"""Library-GEMM layout study for the Llama-2-7B linears on one MI355X.

For every linear (tokens M=8192) times the three training GEMMs — forward
Y = X W^T, dgrad dX = dY W, wgrad dW += dY^T X (fp32 accumulate in place) —
in the candidate call forms, on random bf16 data.  Prints TFLOP/s per form.
"""
import argparse
import json
import time

import torch
import torch.nn.functional as F

SHAPES = {"qkv": (12288, 4096), "dense": (4096, 4096), "fc1": (22016, 4096),
          "fc2": (4096, 11008), "lm_head": (32000, 4096)}


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=8192)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    M = a.M
    res = {}
    torch.manual_seed(0)
    for name, (N, K) in SHAPES.items():
        X = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        W = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        Wt = W.t().contiguous()
        dY = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        G = torch.zeros(N, K, device="cuda", dtype=torch.float32)
        Gt = torch.zeros(K, N, device="cuda", dtype=torch.float32)
        fl = 2.0 * M * N * K
        dYt = dY.t().contiguous()
        Xt = X.t().contiguous()
        forms = {
            "fwd_matmul_WT": lambda: torch.matmul(X, W.t()),
            "fwd_linear": lambda: F.linear(X, W),
            "fwd_matmul_Wt_stored": lambda: torch.matmul(X, Wt),
            "dgrad_matmul_W": lambda: torch.matmul(dY, W),
            "dgrad_matmul_Wt_stored": lambda: torch.matmul(dY, Wt.t()),
            "wgrad_addmm_fp32": lambda: torch.addmm(G, dY.t(), X, out_dtype=torch.float32, out=G),
            "wgrad_addmm_fp32_T": lambda: torch.addmm(Gt, X.t(), dY, out_dtype=torch.float32, out=Gt),
            "wgrad_mm_bf16": lambda: torch.mm(dY.t(), X),
            # token-contiguous (pre-transposed) operands: K-contiguous on both sides
            "wgrad_TN_fp32": lambda: torch.addmm(G, dYt, Xt.t(), out_dtype=torch.float32, out=G),
            "wgrad_TN_bf16": lambda: torch.mm(dYt, Xt.t()),
        }
        copies = {
            "transpose_X_us": lambda: X.t().contiguous(),
            "transpose_dY_us": lambda: dY.t().contiguous(),
        }
        res[name] = {}
        for fname, fn in forms.items():
            try:
                dt = bench(fn)
                res[name][fname] = round(fl / dt / 1e12, 1)
            except Exception as e:  # pragma: no cover
                res[name][fname] = f"err: {str(e)[:80]}"
        for cname, fn in copies.items():
            res[name][cname] = round(bench(fn) * 1e6, 1)
        print(name, json.dumps(res[name]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

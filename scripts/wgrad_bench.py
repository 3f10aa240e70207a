"""Custom MFMA wgrad GEMM (csrc/gemm_wgrad.hip) vs hipBLASLt: numerics + TFLOP/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402

SHAPES = {"qkv": (12288, 4096), "dense": (4096, 4096), "fc1": (22016, 4096),
          "fc2": (4096, 11008), "lm_head": (32000, 4096)}


def _time(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def check():
    C = ext()
    torch.manual_seed(0)
    for (M, N, K) in [(32, 256, 256), (96, 256, 512), (128, 256, 256), (256, 512, 768), (1024, 768, 512), (8192, 512, 256)]:
        dY = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        X = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        G = torch.randn(N, K, device="cuda", dtype=torch.float32)
        ref = G + dY.float().t() @ X.float()
        C.wgrad_gemm(dY, X, G, True)
        err = (G - ref).abs().max().item()
        G2 = torch.full((N, K), float("nan"), device="cuda")
        C.wgrad_gemm(dY, X, G2, False)
        err2 = (G2 - (dY.float().t() @ X.float())).abs().max().item()
        print(f"check M={M} N={N} K={K}: max err accum {err:.3e} store {err2:.3e}", flush=True)
        assert err < 1e-2 and err2 < 1e-2


def main():
    check()
    C = ext()
    M = 16384  # tokens of one 7B micro-batch (16 x 1024)
    out = {}
    for name, (N, K) in SHAPES.items():
        dY = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        X = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        G = torch.zeros(N, K, device="cuda", dtype=torch.float32)
        fl = 2.0 * M * N * K
        t_ours = _time(lambda: C.wgrad_gemm(dY, X, G, True))
        t_lt = _time(lambda: C.lt_gemm(dY, True, X, False, G, 1.0, 1.0, -1))
        t_torch = _time(lambda: torch.addmm(G, dY.t(), X, out_dtype=torch.float32, out=G))
        out[name] = {"ours_tflops": round(fl / t_ours / 1e12, 1),
                     "hipblaslt_default_tflops": round(fl / t_lt / 1e12, 1),
                     "torch_addmm_tflops": round(fl / t_torch / 1e12, 1)}
        print(name, json.dumps(out[name]), flush=True)
        del dY, X, G
    if len(sys.argv) > 1 and sys.argv[1].endswith(".json"):
        json.dump(out, open(sys.argv[1], "w"), indent=1)




def variants(rounds=3):
    """Interleaved A/B (one process, CDNA guide rule 24) of the persistent 4-wave
    kernel, the 8-wave ping-pong kernel and hipBLASLt on the 7B wgrad shapes."""
    import statistics
    C = ext()
    M = 16384
    res = {}
    for name, (N, K) in SHAPES.items():
        dY = torch.rand(M, N, device="cuda", dtype=torch.bfloat16) - 0.5
        X = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) - 0.5
        G = torch.zeros(N, K, device="cuda", dtype=torch.float32)
        fl = 2.0 * M * N * K
        r = {"v4": [], "v8": [], "lt": []}
        for _ in range(rounds):
            for v in (4, 8):
                C.wgrad_set_variant(v)
                r[f"v{v}"].append(fl / _time(lambda: C.wgrad_gemm(dY, X, G, True)) / 1e12)
            C.wgrad_set_variant(4)
            r["lt"].append(fl / _time(lambda: C.lt_gemm(dY, True, X, False, G, 1.0, 1.0, -1)) / 1e12)
        res[name] = {k: round(statistics.median(v), 1) for k, v in r.items()}
        print(f"{name:8s} v4 {res[name]['v4']:7.1f}  v8 {res[name]['v8']:7.1f}  hipBLASLt "
              f"{res[name]['lt']:7.1f} TF/s  (v4/v8 x{res[name]['v4'] / res[name]['v8']:.3f})",
              flush=True)
        del dY, X, G
    return res


if __name__ == "__main__":
    if "--variants" in sys.argv:
        variants()
    else:
        main()

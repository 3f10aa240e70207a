"""A/B of bench-only GEMM builds (scripts/lab/gemm_lab.hip) against the production
persistent NT kernel and hipBLASLt: interleaved timing in one process (CDNA
guide rule 24), uniform-random bf16 operands, median over rounds.  Variant 1
is also checked against hipBLASLt's output.

    python -m epfl_megatron_amd.build --lab     # once, on the CPU: scripts/lab/_gemm_lab.so
    python scripts/gemm_lab.py [M N K ...]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.ops._ext import ext  # noqa: E402


def _lab():
    import importlib.util
    so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lab", "_gemm_lab.so")
    if not os.path.exists(so):
        raise SystemExit("build the lab first: python -m epfl_megatron_amd.build --lab")
    spec = importlib.util.spec_from_file_location("_gemm_lab", so)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


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
    L = _lab()
    C.gemm_nt_set_variant(6)  # production = the persistent kernel
    args = [int(v) for v in sys.argv[1:]]
    shapes = [tuple(args[i:i + 3]) for i in range(0, len(args), 3)] or \
        [(16384, 4096, 4096), (16384, 4096, 11008), (16384, 11008, 4096), (16384, 12288, 4096)]
    variants = [int(v) for v in os.environ.get("LAB_VARIANTS", "0,1").split(",")]
    for M, N, K in shapes:
        a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ref = torch.matmul(a, b.t())
        for v in variants:
            c.zero_()
            L.gemm_lab(a, b, c, v)
            err = ((c.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
            assert err < 2e-2, f"variant {v} wrong: rel err {err}"
        fl = 2.0 * M * N * K
        r = {f"lab{v}": [] for v in variants}
        r["prod"] = []
        r["hipblaslt"] = []
        for _ in range(5):
            for v in variants:
                r[f"lab{v}"].append(fl / _t(lambda: L.gemm_lab(a, b, c, v)) / 1e12)
            r["prod"].append(fl / _t(lambda: C.gemm_nt(a, b, c)) / 1e12)
            r["hipblaslt"].append(fl / _t(lambda: torch.matmul(a, b.t(), out=c)) / 1e12)
        print(f"M={M} N={N} K={K}: " + "  ".join(
            f"{k} {statistics.median(v):7.1f}" for k, v in r.items()) + " TF/s", flush=True)


if __name__ == "__main__":
    main()

"""Cost of splitting the SP GEMMs into pieces (1 GPU, no communication):
the monolithic GEMM of a TP rank vs the same product as c pieces through the
row-group remaps of sp_allgather_gemm / sp_gemm_reducescatter
(parallel/tensor/layers.py).  Shapes: one TP=8 rank of Llama-2-7B at seq 4096,
micro-batch 4 (16k token rows).

    python scripts/sp_overlap_bench.py [--tokens 16384] [--tp 8] [--chunks 2]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--chunks", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from epfl_megatron_amd.ops._ext import ext
    C = ext()
    dt, dev = torch.bfloat16, "cuda"
    M, tp, c = a.tokens, a.tp, a.chunks
    R = M // tp // c
    H, F, Q = 4096, 11008 // tp, 3 * 4096 // tp

    def r(*s):
        return torch.empty(*s, device=dev, dtype=dt).uniform_(-1, 1)

    cases = []
    # all-gather side (QKV, fc1 + GLU): the pieces write through c_map
    for name, n in (("qkv", Q),):
        x, w, out = r(M, H), r(n, H), torch.empty(M, n, device=dev, dtype=dt)
        g = [x[j * tp * R:(j + 1) * tp * R] for j in range(c)]
        cases.append((name, 2.0 * M * n * H, lambda x=x, w=w, out=out: C.gemm_nt(x, w, out),
                      lambda g=g, w=w, out=out: [C.gemm_nt(g[j], w, out, [], [R, c * R, j * R])
                                                 for j in range(c)]))
    x, w1 = r(M, H), r(2 * F, H)
    pre, y = torch.empty(M, 2 * F, device=dev, dtype=dt), torch.empty(M, F, device=dev, dtype=dt)
    g = [x[j * tp * R:(j + 1) * tp * R] for j in range(c)]
    cases.append(("fc1+glu", 2.0 * M * 2 * F * H,
                  lambda x=x, w1=w1, pre=pre, y=y: C.gemm_nt_glu(x, w1, 0, pre, y, []),
                  lambda g=g, w1=w1, pre=pre, y=y: [C.gemm_nt_glu(g[j], w1, 0, pre, y, [R, c * R, j * R])
                                                    for j in range(c)]))
    # piece-major GLU MLP (layers._sp_mlp_forward): every piece a plain product
    # into its own contiguous buffer, no row remap
    prep = torch.empty(c, tp * R, 2 * F, device=dev, dtype=dt)
    yp = torch.empty(c, tp * R, F, device=dev, dtype=dt)
    cases.append(("fc1+glu piece-major", 2.0 * M * 2 * F * H,
                  lambda x=x, w1=w1, pre=pre, y=y: C.gemm_nt_glu(x, w1, 0, pre, y, []),
                  lambda g=g, w1=w1, prep=prep, yp=yp: [C.gemm_nt_glu(g[j], w1, 0, prep[j], yp[j], [])
                                                        for j in range(c)]))
    # the MLP pipeline's own piece sizes (layers._sp_mlp_pieces: uneven where
    # even pieces quantize the fc1 + GLU tiles), piece-major, no row remap
    # (the tile-round plan of round 4: 23 + 41 tile rows of 256; the pipeline
    # keeps even pieces, see layers._sp_mlp_pieces)
    m1 = 256 // -(-2 * F // 256) * 256 // tp
    sizes = [m1, M // tp - m1]
    offs = [sum(sizes[:j]) for j in range(len(sizes))]
    gu = [x[tp * o:tp * (o + n)] for o, n in zip(offs, sizes)]
    preu = [prep.view(-1, 2 * F)[tp * o:tp * (o + n)] for o, n in zip(offs, sizes)]
    yu = [yp.view(-1, F)[tp * o:tp * (o + n)] for o, n in zip(offs, sizes)]
    cases.append((f"fc1+glu planned pieces {sizes}", 2.0 * M * 2 * F * H,
                  lambda x=x, w1=w1, pre=pre, y=y: C.gemm_nt_glu(x, w1, 0, pre, y, []),
                  lambda gu=gu, w1=w1, preu=preu, yu=yu: [C.gemm_nt_glu(a, w1, 0, b_, c_, [])
                                                          for a, b_, c_ in zip(gu, preu, yu)]))
    w2 = r(H, F)
    yfull = r(M, F)
    o2 = torch.empty(M, H, device=dev, dtype=dt)
    partp = torch.empty(c, tp * R, H, device=dev, dtype=dt)
    cases.append(("fc2 piece-major", 2.0 * M * H * F,
                  lambda y=yfull, w2=w2, o2=o2: C.gemm_nt(y, w2, o2),
                  lambda y=yfull, w2=w2, partp=partp: [C.gemm_nt(y[j * tp * R:(j + 1) * tp * R], w2,
                                                                 partp[j]) for j in range(c)]))
    # the whole MLP forward (fc1 + GLU, fc2) as the pipeline runs it: even
    # pieces vs the planned ones
    o2b = torch.empty(M, H, device=dev, dtype=dt)

    def mlp(parts, x=x, w1=w1, w2=w2, pre=pre, y=y, o2b=o2b):
        for o, n in parts:
            rows = slice(tp * o, tp * (o + n))
            C.gemm_nt_glu(x[rows], w1, 0, pre[rows], y[rows], [])
            C.gemm_nt(y[rows], w2, o2b[rows])
    even = [(j * R, R) for j in range(c)]
    cases.append((f"mlp fwd planned {sizes} vs even", 2.0 * M * 3 * F * H,
                  lambda: mlp(even), lambda: mlp(list(zip(offs, sizes)))))
    # reduce-scatter side (attention out, fc2): the pieces read through a_map
    for name, k in (("o_proj", H // tp), ("fc2", F)):
        x, w = r(M, k), r(H, k)
        out = torch.empty(M, H, device=dev, dtype=dt)
        part = torch.empty(c, tp * R, H, device=dev, dtype=dt)
        cases.append((name, 2.0 * M * H * k, lambda x=x, w=w, out=out: C.gemm_nt(x, w, out),
                      lambda x=x, w=w, part=part: [C.gemm_nt(x, w, part[j], [R, c * R, j * R], [],
                                                             tp * R) for j in range(c)]))
    res = {n: {"mono": [], "pieces": []} for n, *_ in cases}
    for _ in range(a.rounds):
        for name, fl, mono, pieces in cases:
            res[name]["mono"].append(timeit(mono))
            res[name]["pieces"].append(timeit(pieces))
    out = {}
    for name, fl, _, _ in cases:
        m, p = statistics.median(res[name]["mono"]), statistics.median(res[name]["pieces"])
        out[name] = {"mono_ms": round(m, 4), "pieces_ms": round(p, 4),
                     "mono_tflops": round(fl / m / 1e9, 1), "pieces_tflops": round(fl / p / 1e9, 1),
                     "pieces_over_mono": round(p / m, 4)}
        print(f"{name:8s} monolithic {m:7.4f} ms ({fl / m / 1e9:6.1f} TF/s)   {c} pieces "
              f"{p:7.4f} ms ({fl / p / 1e9:6.1f} TF/s)   ratio {p / m:.3f}", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"tokens": M, "tp": tp, "chunks": c, "cases": out}, f, indent=1)


if __name__ == "__main__":
    main()

"""Context-parallel document-mask pair kernels vs the fp32 CPU path of the same
pair (parallel/context.py): one pair at a time, diagonal (causal, offset 0)
and off-diagonal (causal kernel with offset sk), forward (fused merge form,
merge off) and backward.  Prints max error / NaN count per case.
Usage: python scripts/cp_doc_debug.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from epfl_megatron_amd.parallel import context as C  # noqa: E402
from epfl_megatron_amd.utils.misc import doc_bounds  # noqa: E402


def case(name, n, pq0, pk0, causal, coff, nq=8, nkv=2, hd=128, seed=0):
    torch.manual_seed(seed)
    b, S = 2, 4 * n
    tok = torch.randint(1, 100, (b, S))
    for i in range(b):
        tok[i, torch.randperm(S - 1)[:3 + 2 * i]] = 0
    docs = doc_bounds(tok, 0)
    pq = torch.arange(pq0, pq0 + n)
    pk = torch.arange(pk0, pk0 + n)
    pd = C._pair_docs(docs, pq, pk)
    q = torch.randn(b, n, nq, hd, dtype=torch.bfloat16)
    k = torch.randn(b, n, nkv, hd, dtype=torch.bfloat16)
    v = torch.randn(b, n, nkv, hd, dtype=torch.bfloat16)
    do = torch.randn(b, n, nq, hd, dtype=torch.bfloat16)
    o_ref, lse_ref = C._pair_fwd(q, k, v, causal, hd ** -0.5, pd, coff)
    dev = "cuda"
    qg, kg, vg = q.to(dev), k.to(dev), v.to(dev)
    o = torch.empty(b, n, nq, hd, dtype=torch.float32, device=dev)
    lse = torch.empty(b, nq, n, dtype=torch.float32, device=dev)
    C._pair_fwd_into(qg, kg, vg, o, lse, causal, hd ** -0.5, False, pd.to(dev), coff)
    torch.cuda.synchronize()
    fin = torch.isfinite(lse_ref)
    eo = (o.cpu() - o_ref).abs()
    el = (lse.cpu() - lse_ref).abs()[fin]
    print(f"{name} fwd: o max err {eo.nan_to_num(99).max().item():.3e} nan {torch.isnan(o).sum().item()} "
          f"| lse max err {el.max().item() if el.numel() else 0:.3e} rows-without-keys "
          f"{(~fin).sum().item()} gpu-lse-of-those {lse.cpu()[~fin][:4].tolist()}", flush=True)
    # backward with the reference o / lse (finite rows only matter)
    lse_g = lse_ref.clone()
    lse_g[~fin] = 0.0
    dq_r, dk_r, dv_r = C._pair_bwd(q, k, v, o_ref.to(torch.bfloat16), lse_g, do, causal, hd ** -0.5,
                                   pd, coff)
    dq, dk, dv = C._pair_bwd(qg, kg, vg, o_ref.to(torch.bfloat16).to(dev), lse_g.to(dev), do.to(dev),
                             causal, hd ** -0.5, pd.to(dev), coff)
    torch.cuda.synchronize()
    for nm, a, r in (("dq", dq, dq_r), ("dk", dk, dk_r), ("dv", dv, dv_r)):
        e = (a.cpu() - r).abs()
        print(f"{name} bwd {nm}: max err {e.nan_to_num(99).max().item():.3e} "
              f"(ref max {r.abs().max().item():.2f}) nan {torch.isnan(a).sum().item()}", flush=True)


if __name__ == "__main__":
    n = 96
    case("diag", n, 0, 0, True, None)
    case("diag-later", n, 2 * n, 2 * n, True, None)
    case("offdiag", n, 2 * n, 0, True, n)
    case("offdiag-adjacent", n, n, 0, True, n)
    case("diag-256", 256, 0, 0, True, None)
    case("offdiag-256", 256, 512, 0, True, 256)

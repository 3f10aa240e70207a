"""Where a FlashAttention forward workgroup spends its time (diagnostics).

Runs the forward with per-workgroup wall-clock stamps (csrc/flash_attn_fwd.hip,
AttnParams::stamps: s_memrealtime, 10 ns) and reports, per shape, the median
prologue (entry -> first K/V tiles landed), loop, epilogue (O / LSE stores
drained) and the gap between consecutive workgroups on the same CU.

    python scripts/fa_stamps.py [--json out.json]
"""
import argparse
import collections
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(C, b, s, nq, hd, causal):
    q = torch.empty(b, s, nq, hd, device="cuda", dtype=torch.bfloat16).uniform_(-2, 2)
    k = torch.empty_like(q).uniform_(-2, 2)
    v = torch.empty_like(q).uniform_(-1, 1)
    out = torch.empty_like(q)
    lse = torch.empty(b, nq, s, device="cuda", dtype=torch.float32)
    qs = [q.stride(0), q.stride(1), q.stride(2), q.stride(2)]
    ks = [k.stride(0), k.stride(1), k.stride(2)]
    os_ = [out.stride(0), out.stride(1), out.stride(2)]

    def call():
        C.flash_attn_fwd(q, k, v, out, lse, b, s, s, nq, nq, hd, qs, ks, ks, os_, causal,
                         hd ** -0.5, None, None, None, None)

    # block rows: 32 per wave, 4 waves when the 8-wave grid is under 512
    # blocks (csrc/flash_attn_fwd.hip flash_attn_waves)
    blocks8 = ((s + 255) // 256) * nq * b
    bm = 128 if blocks8 < 512 else 256
    nblk = ((s + bm - 1) // bm) * nq * b
    buf = torch.zeros(nblk * 8 + 4096, dtype=torch.int64, device="cuda")
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    C.fa_set_stamps(buf)
    call()
    torch.cuda.synchronize()
    C.fa_set_stamps(None)
    st = buf[:nblk * 8].view(nblk, 8).cpu().tolist()
    t0 = min(r[0] for r in st)
    pro = [(r[1] - r[0]) * 10e-3 for r in st]
    loop = [(r[2] - r[1]) * 10e-3 for r in st]
    epi = [(r[3] - r[2]) * 10e-3 for r in st]
    span = (max(r[3] for r in st) - t0) * 10e-3
    per_cu = collections.defaultdict(list)
    for r in st:
        per_cu[(r[5], r[4])].append(r)
    gaps, nper = [], []
    for rows in per_cu.values():
        rows.sort(key=lambda r: r[0])
        nper.append(len(rows))
        for a, bb in zip(rows, rows[1:]):
            gaps.append((bb[0] - a[3]) * 10e-3)
    busy = sum((r[3] - r[0]) for r in st) * 10e-3 / max(1, len(per_cu))
    # causal balance: each CU's last end, and the query blocks it ran (mb =
    # nmb - 1 - lin / (nq * b): heaviest first)
    ends = sorted((max(r[3] for r in rows) - t0) * 10e-3 for rows in per_cu.values())
    nmb = (s + bm - 1) // bm
    idx = {id(r): i for i, r in enumerate(st)}
    mbs = sorted((sorted(nmb - 1 - idx[id(r)] // (nq * b) for r in rows) for rows in per_cu.values()),
                 key=lambda m: -sum(m))
    med = statistics.median
    rec = {"b": b, "s": s, "causal": causal, "blocks": nblk, "cus": len(per_cu),
           "span_us": round(span, 1), "busy_us_per_cu": round(busy, 1),
           "prologue_us_med": round(med(pro), 2), "loop_us_med": round(med(loop), 2),
           "epilogue_us_med": round(med(epi), 2),
           "gap_us_med": round(med(gaps), 2) if gaps else None,
           "gap_us_p90": round(sorted(gaps)[int(0.9 * len(gaps))], 2) if gaps else None,
           "blocks_per_cu_min_max": [min(nper), max(nper)],
           "last_start_us": round((max(r[0] for r in st) - t0) * 10e-3, 1),
           "nq": nq, "block_rows": bm,
           "cu_end_us_min_med_max": [round(ends[0], 1), round(ends[len(ends) // 2], 1),
                                     round(ends[-1], 1)],
           "cu_qblocks_heaviest": mbs[:3], "cu_qblocks_lightest": mbs[-3:]}
    print(json.dumps(rec), flush=True)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    from epfl_megatron_amd.ops._ext import ext
    C = ext()
    res = []
    for (b, s) in ((16, 1024), (4, 4096)):
        for causal in (False, True):
            res.append(run(C, b, s, 32, 128, causal))
    # one TP rank of Llama-2-7B at TP = 8 (4 heads), the proxy's attention
    res.append(run(C, 4, 4096, 4, 128, True))
    # Llama-2-70B at TP = 8 (8 heads per rank, micro-batch 1): one 4-wave block per CU
    res.append(run(C, 1, 4096, 8, 128, True))
    if args.json:
        json.dump(res, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()

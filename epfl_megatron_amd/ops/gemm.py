"""Tuned hipBLASLt GEMMs for the three training products of every linear layer.

    forward  Y[M,N]  = X[M,K] @ W[N,K]^T          (bf16 out)
    dgrad    dX[M,K] = dY[M,N] @ W[N,K]           (bf16 out)
    wgrad    G[N,K] (+)= dY[M,N]^T @ X[M,K]       (fp32 main_grad, beta 1 or 0)

PyTorch calls hipBLASLt with its first heuristic solution.  On MI355X that
choice is 5-30 % slower than the best solution for these shapes
(profiles/r1_lt_tune.json), and TunableOp does not cover the fp32-output
wgrad.  Here the first call of each (product, M, N, K, dtype) times the
heuristic top candidates on the live device, in-process and back to back (so
DVFS / device-to-device variance cancels), and keeps the fastest solution
index; later calls go straight to ``_C.lt_gemm``.  Results persist in a
small JSON cache (``EMA_GEMM_CACHE``, default ``~/.cache/epfl_megatron_amd``)
keyed by device name and hipBLASLt build.  ``EMA_GEMM_TUNE=0`` disables
tuning (heuristic solution, same call path).
"""
import json
import os
import threading

import torch

from ._ext import ext

_LOCK = threading.Lock()
_BEST = {}
_LOADED = False
_CANDIDATES = int(os.environ.get("EMA_GEMM_CANDIDATES", "24"))
_TUNE = os.environ.get("EMA_GEMM_TUNE", "1") != "0"


def _cache_path():
    d = os.environ.get("EMA_GEMM_CACHE",
                       os.path.join(os.path.expanduser("~"), ".cache", "epfl_megatron_amd"))
    return os.path.join(d, "gemm_tune.json")


def _device_tag():
    p = torch.cuda.get_device_properties(torch.cuda.current_device())
    return f"{p.name}|{getattr(p, 'gcnArchName', '')}|{torch.version.hip}"


def _load():
    global _LOADED
    if _LOADED:
        return
    _LOADED = True
    try:
        with open(_cache_path()) as f:
            data = json.load(f)
        _BEST.update(data.get(_device_tag(), {}))
    except (OSError, ValueError):
        pass


def _save():
    path = _cache_path()
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        try:
            with open(path) as f:
                data = json.load(f)
        except (OSError, ValueError):
            data = {}
        data[_device_tag()] = dict(_BEST)
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump(data, f)
        os.replace(tmp, path)
    except OSError:
        pass


def _time(fn, iters=3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e)


def _tune(key, P, tp, Q, tq, D, beta):
    """Pick the fastest solution; operands are scratch copies (D is clobbered)."""
    C = ext()
    algos = C.lt_algos(P, tp, Q, tq, D, beta, _CANDIDATES)[:_CANDIDATES]
    best, best_t = -1, None
    for a in [-1] + algos:
        try:
            C.lt_gemm(P, tp, Q, tq, D, 1.0, beta, a)  # warm / validate
            t = _time(lambda: C.lt_gemm(P, tp, Q, tq, D, 1.0, beta, a))
        except RuntimeError:
            continue
        if best_t is None or t < best_t:
            best, best_t = a, t
    return best


def _algo(kind, P, tp, Q, tq, D, beta):
    M = D.shape[0]
    key = f"{kind}:{M}x{D.shape[1]}x{P.shape[0] if tp else P.shape[1]}:{P.dtype}"
    a = _BEST.get(key)
    if a is not None:
        return a
    with _LOCK:
        _load()
        a = _BEST.get(key)
        if a is not None:
            return a
        if not _TUNE:
            _BEST[key] = -1
            return -1
        # tune on scratch tensors of the same shapes (never clobber live data)
        scratch_d = torch.empty_like(D)
        if beta:
            scratch_d.zero_()
        a = _tune(key, P, tp, Q, tq, scratch_d, beta)
        del scratch_d
        _BEST[key] = a
        _save()
        return a


def _ok(*ts):
    return all(t.is_cuda and t.dim() == 2 and t.stride(1) == 1 for t in ts)


def linear_fwd(x2d, w):
    """Y = X W^T (bf16/fp16 in and out)."""
    if not _ok(x2d, w) or x2d.dtype not in (torch.bfloat16, torch.float16):
        return torch.matmul(x2d, w.t())
    y = torch.empty(x2d.shape[0], w.shape[0], device=x2d.device, dtype=x2d.dtype)
    ext().lt_gemm(x2d, False, w, True, y, 1.0, 0.0, _algo("fwd", x2d, False, w, True, y, 0.0))
    return y


def linear_dgrad(dy2d, w):
    """dX = dY W."""
    if not _ok(dy2d, w) or dy2d.dtype not in (torch.bfloat16, torch.float16):
        return torch.matmul(dy2d, w)
    dx = torch.empty(dy2d.shape[0], w.shape[1], device=dy2d.device, dtype=dy2d.dtype)
    ext().lt_gemm(dy2d, False, w, False, dx, 1.0, 0.0,
                  _algo("dgrad", dy2d, False, w, False, dx, 0.0))
    return dx


def wgrad(main_grad2d, dy2d, x2d, accumulate):
    """main_grad (+)= dY^T X into the fp32 buffer in place."""
    beta = 1.0 if accumulate else 0.0
    if not _ok(main_grad2d, dy2d, x2d):
        torch.addmm(main_grad2d, dy2d.t(), x2d, beta=beta, out_dtype=torch.float32,
                    out=main_grad2d)
        return
    ext().lt_gemm(dy2d, True, x2d, False, main_grad2d, 1.0, beta,
                  _algo("wgrad", dy2d, True, x2d, False, main_grad2d, beta))

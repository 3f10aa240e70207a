"""One-shot xGMI all-reduce / all-gather (csrc/xgmi_allreduce.hip, parallel/xgmi.py).

Several processes share the one GPU of the test box: each maps the others'
regions through same-device IPC handles, so the flag / parity protocol and the
kernel are the ones a multi-GPU TP group runs (the transport there is xGMI).
Oracle: the fp32 sum of every rank's input in rank order, rounded once to the
dtype (the kernel's exact arithmetic), and bitwise equality across ranks.
"""
import pytest
import torch

from dist_utils import run_dist

pytestmark = pytest.mark.gpu

DTYPES = (torch.bfloat16, torch.float16, torch.float32)


def _inputs(world, n, dt, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(n, generator=g).to(dt) for _ in range(world)]


def _oracle(xs):
    acc = torch.zeros(xs[0].shape, dtype=torch.float32)
    for x in xs:
        acc += x.float()
    return acc.to(xs[0].dtype)


def _rank(rank, world):
    import torch.distributed as dist

    from epfl_megatron_amd.parallel import comm
    from epfl_megatron_amd.parallel.xgmi import XgmiAllReduce

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    xg = XgmiAllReduce(None, cap_bytes=256 * 1024)
    bad = []
    # sizes: one partial chunk, a chunk boundary + tail, many chunks; 30 rounds
    # cycle the epochs through both parities many times
    for it in range(30):
        for dt in DTYPES:
            for n in (8, 2048 + 8, 40000):
                xs = _inputs(world, n, dt, 1000 * it + n)
                t = xs[rank].cuda()
                if it % 2:
                    xg(t)
                    got = t
                else:
                    got = torch.empty_like(t)
                    xg(t, got)
                torch.cuda.synchronize()
                if not torch.equal(got.cpu(), _oracle(xs)):
                    bad.append((it, str(dt), n))
    xg.check()
    # all-gather (rank-major along dim 0): out of place and in place
    for it in range(6):
        for dt in DTYPES:
            n = (8, 2048 + 8, 40000)[it % 3]
            xs = _inputs(world, n, dt, 500 + 31 * it + n)
            ref = torch.cat(xs)
            out = torch.empty(world * n, dtype=dt, device="cuda")
            if it % 2:
                out.view(world, n)[rank].copy_(xs[rank])
                xg.all_gather(out, out.view(world, n)[rank])
            else:
                xg.all_gather(out, xs[rank].cuda())
            torch.cuda.synchronize()
            if not torch.equal(out.cpu(), ref):
                bad.append(("gather", it, str(dt), n))
    xg.check()
    # captured in a hipGraph: replays advance the device-side epochs
    t = torch.zeros(4096, dtype=torch.bfloat16, device="cuda")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        xg(t)
    for rep in range(5):
        xs = _inputs(world, 4096, torch.bfloat16, 77 + rep)
        t.copy_(xs[rank])
        g.replay()
        torch.cuda.synchronize()
        if not torch.equal(t.cpu(), _oracle(xs)):
            bad.append(("graph", rep))
    xg.check()
    # latency of an 8 KiB call (ranks sharing the GPU: an upper bound on the
    # kernel's own cost, with no xGMI hop in it): eager and graph-replayed
    import time
    for _ in range(20):
        xg(t)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(200):
        xg(t)
    torch.cuda.synchronize()
    eager_us = (time.perf_counter() - t0) / 200 * 1e6
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(200):
        g.replay()
    torch.cuda.synchronize()
    graph_us = (time.perf_counter() - t0) / 200 * 1e6
    xg.check()
    if rank == 0:
        print(f"xgmi one-shot 8 KiB bf16, world {world} on one GPU: eager {eager_us:.1f} us/call, "
              f"graph replay {graph_us:.1f} us/call", flush=True)
    # routing through comm.all_reduce: small sum -> one-shot kernel, the rest
    # (too large for the registered capacity) -> the process group
    grp = dist.group.WORLD
    comm._XGMI[id(grp)] = xg
    comm.report(reset=True)
    xs = _inputs(world, 1024, torch.float32, 5)
    t = xs[rank].cuda()
    comm.all_reduce(t, group=grp)
    big = torch.ones(128 * 1024, dtype=torch.float32, device="cuda")
    comm.all_reduce(big, group=grp)
    gout = torch.empty(world * 512, dtype=torch.bfloat16, device="cuda")
    comm.all_gather_into(gout, torch.full((512,), float(rank), dtype=torch.bfloat16, device="cuda"),
                         group=grp)
    torch.cuda.synchronize()
    rep = comm.report()
    routed = [k for k in rep if k.startswith("all_reduce_xgmi")]
    routed_g = [k for k in rep if k.startswith("all_gather_xgmi")]
    gref = torch.arange(world).repeat_interleave(512).to(torch.bfloat16)
    if not routed_g or not torch.equal(gout.cpu(), gref):
        bad.append(("comm gather", sorted(rep)))
    if not torch.equal(t.cpu(), _oracle(xs)) or not routed or not torch.all(big == world):
        bad.append(("comm", sorted(rep)))
    comm._XGMI.pop(id(grp))
    xg.check()
    out = (bad, t.cpu())
    dist.barrier()
    xg.close()
    return out


def _rank_sp_gather(rank, world):
    """(2 ranks: their two 1024-workgroup grids must be co-resident on the one
    GPU of the test box; across GPUs there is no such limit.)
    Multi-MiB all-gathers of sequence-parallel [s/tp, b, h] pieces through
    the one-shot kernel (separate gather cap), checked against the process
    group's own all_gather_into_tensor; misaligned tensors are staged (the
    routing decision never depends on an address)."""
    import torch.distributed as dist

    from epfl_megatron_amd.parallel import comm
    from epfl_megatron_amd.parallel.xgmi import XgmiAllReduce

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    grp = dist.group.WORLD
    xg = XgmiAllReduce(grp, cap_bytes=64 * 1024, gather_cap_bytes=4 * 1024 * 1024)
    comm._XGMI[id(grp)] = xg
    bad = []
    g = torch.Generator().manual_seed(11 + rank)
    for it, (s, b, h) in enumerate(((512, 1, 4096), (256, 2, 2048), (128, 1, 4096))):
        piece = torch.randn(s, b, h, generator=g).to(torch.bfloat16)
        ref = torch.empty(world * s, b, h, dtype=torch.bfloat16)
        dist.all_gather_into_tensor(ref, piece, group=grp)  # gloo oracle
        out = torch.empty(world * s, b, h, dtype=torch.bfloat16, device="cuda")
        comm.report(reset=True)
        comm.all_gather_into(out, piece.cuda(), group=grp)
        torch.cuda.synchronize()
        rep = comm.report()
        if not any(k.startswith("all_gather_xgmi") for k in rep):
            bad.append(("not routed", it, sorted(rep)))
        if not torch.equal(out.cpu(), ref):
            bad.append(("sp gather", it))
    # all-reduce above its own cap goes to the process group even though the
    # registered region is larger (the gather cap)
    big = torch.ones(256 * 1024, dtype=torch.float32, device="cuda")
    comm.report(reset=True)
    comm.all_reduce(big, group=grp)
    torch.cuda.synchronize()
    if any(k.startswith("all_reduce_xgmi") for k in comm.report()) or not torch.all(big == world):
        bad.append("all-reduce cap")
    # a tensor at an odd byte offset (rank-dependent alignment) is staged
    raw = torch.zeros(4096 + 8 * rank + 1, dtype=torch.bfloat16, device="cuda")
    t = raw[1 + 8 * rank: 1 + 8 * rank + 4096]
    t.fill_(float(rank + 1))
    comm.all_reduce(t, group=grp)
    torch.cuda.synchronize()
    if not torch.all(t.cpu() == float(sum(range(1, world + 1)))):
        bad.append("misaligned all-reduce")
    comm._XGMI.pop(id(grp))
    xg.check()
    dist.barrier()
    xg.close()
    return bad


def _rank_dead_peer(rank, world):
    """Rank 1 never joins: rank 0's call ends after EMA_XGMI_TIMEOUT_MS with a
    NaN-filled output, and check() raises (no hang, no stale sums)."""
    import time

    import torch.distributed as dist

    from epfl_megatron_amd.parallel.xgmi import XgmiAllReduce, XgmiError

    from epfl_megatron_amd.parallel import comm

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    # a short per-communicator bound (what a decode server may choose); the
    # default is long (test_xgmi_slow_peer_is_not_a_timeout)
    xg = XgmiAllReduce(None, cap_bytes=64 * 1024, timeout_ms=300)
    res = None
    if rank == 0:
        t = torch.ones(8192, dtype=torch.bfloat16, device="cuda")
        t0 = time.perf_counter()
        xg(t)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        # the device error word folds into the grad-norm square: the step is
        # skipped on device (comm.fold_xgmi_error), no host sync needed
        comm._XGMI[id(None)] = xg
        try:
            folded = comm.fold_xgmi_error(torch.tensor([4.0], device="cuda")).item()
        finally:
            comm._XGMI.pop(id(None), None)
        try:
            xg.check()
            raised = False
        except XgmiError:
            raised = True
        res = (bool(torch.isnan(t.float()).all().item()), raised, dt, folded, xg.timeout_ms)
    dist.barrier()
    xg.close()
    return res


def _rank_slow_peer(rank, world):
    """Rank 1 arrives 2.5 s late (host work: a checkpoint write, a GC pause):
    with the default bound the call completes correctly on both ranks and
    nothing is flagged."""
    import time

    import torch.distributed as dist

    from epfl_megatron_amd.parallel.xgmi import XgmiAllReduce

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    xg = XgmiAllReduce(None, cap_bytes=64 * 1024)
    dist.barrier()
    if rank == 1:
        time.sleep(2.5)
    t = torch.full((8192,), float(rank + 1), dtype=torch.bfloat16, device="cuda")
    xg(t)
    torch.cuda.synchronize()
    ok = bool((t.float() == 3.0).all().item())
    err = int(xg.error_tensor().item())
    xg.check()
    dist.barrier()
    xg.close()
    return ok, err, xg.timeout_ms


def test_xgmi_sp_piece_allgather():
    for bad in run_dist(_rank_sp_gather, 2, timeout=300):
        assert not bad, bad


def test_xgmi_dead_peer_times_out():
    res = run_dist(_rank_dead_peer, 2, timeout=300)
    all_nan, raised, dt, folded, tmo = res[0]
    assert all_nan and raised and tmo == 300
    assert folded == float("inf")  # the optimizer skips the step
    assert dt < 5.0, dt  # bounded by the 300 ms wall-clock wait, not tens of seconds


def test_xgmi_slow_peer_is_not_a_timeout():
    for ok, err, tmo in run_dist(_rank_slow_peer, 2, timeout=300):
        assert ok and err == 0 and tmo == 60000


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_oneshot_allreduce(world):
    res = run_dist(_rank, world, timeout=300)
    for bad, _ in res:
        assert not bad, bad
    # every rank holds the same bits
    for _, t in res[1:]:
        assert torch.equal(t, res[0][1])

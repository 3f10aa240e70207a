"""The one place collectives are issued from.

Every tensor collective the framework runs (TP all-reduce / all-gather /
reduce-scatter, DP bucket reduce-scatter / all-reduce, dist-opt parameter
all-gather) goes through these helpers.  On MI355X they run on RCCL (the
``nccl`` backend name in PyTorch-ROCm) over xGMI; on the CPU plumbing path they
run the *same calls* on ``gloo`` (PyTorch >= 2.10 gloo implements
``reduce_scatter_tensor``, ``all_gather_into_tensor`` and ``ReduceOp.AVG``,
including the in-place forms), so the code the GPU runs is the code the CPU
tests run — there is no backend fork.

Two debug/observability aids live here:

* **per-collective accounting** — every call adds (count, bytes) to a table
  keyed by ``op/group-name``; with ``set_timing(True)`` (``--timing_log_level
  2``) HIP events also measure launch->completion time per op.  ``training.py``
  prints the table at each log interval (``report()``).
* **pipeline p2p** — ``p2p()`` posts one batched isend/irecv group; its bytes
  are accounted per direction (``p2p_send`` / ``p2p_recv``) and, under the race
  checker, a send buffer written before ``wait()`` raises like a collective.
* **in-flight race checker** — ``EMA_COMM_CHECK=1`` turns every async
  collective into "snapshot at launch, verify + run at ``wait()``": if any
  kernel or hook writes the buffer while the collective is logically in
  flight, ``wait()`` raises.  RCCL gives no such guarantee checking, and a
  write into a bucket that is being reduce-scattered silently corrupts
  gradients; the CPU tests run with the checker on.
"""
import os
import time
from collections import OrderedDict

import torch
import torch.distributed as dist

from ..utils import trace as _trace

_CHECK = os.environ.get("EMA_COMM_CHECK", "0") == "1"
_TIMING = [False]
_STATS = OrderedDict()  # key -> [count, bytes, ms]
_GROUP_NAMES = {}
_GROUP_SIZES = {}  # name -> ranks in the group (bus-bandwidth factors of the report)
_PENDING_EVENTS = []  # (key, start_event, end_event) not yet folded into _STATS
_LOOPBACK = {}  # id(group) -> simulated size (--simulated_tensor_parallel_size)
_XGMI = {}  # id(group) -> parallel.xgmi.XgmiAllReduce (one-shot small all-reduce)


class CommRaceError(RuntimeError):
    pass


def set_race_check(enabled):
    global _CHECK
    _CHECK = bool(enabled)


def set_timing(enabled):
    _TIMING[0] = bool(enabled)


def set_loopback(group, world):
    """Make ``group`` (a real 1-rank group) stand for ``world`` ranks: its
    collectives are accounted with a real rank's bytes but move (almost) none,
    so the proxy's timed step holds no emulation kernels a real rank would not
    run: all-gather writes this rank's shard into its
    slot, and into the other ranks' slots too -- every call for a fresh
    output, once per range for a persistent scratch buffer (finite stand-ins
    for the bytes xGMI would deliver, never recycled garbage),
    reduce-scatter writes this rank's own chunk (no reduction), all-reduce /
    broadcast are identities.  Used by the one-GPU per-rank proxies of the TP
    configurations; the numbers they train on are not a real TP run's."""
    if world and world > 1:
        _LOOPBACK[id(group)] = int(world)
    else:
        _LOOPBACK.pop(id(group), None)
    name = _GROUP_NAMES.get(id(group))
    if name is not None and world:
        _GROUP_SIZES[name] = int(world)


def enable_xgmi_allreduce(group, cap_bytes, gather_cap_bytes=None, timeout_ms=None):
    """Route sum all-reduces of at most ``cap_bytes`` and all-gathers of at
    most ``gather_cap_bytes`` per rank (default: ``cap_bytes``) on ``group``
    (contiguous bf16 / fp16 / fp32 CUDA tensors) through the one-shot xGMI
    kernel (``parallel/xgmi.py``); RCCL keeps everything else.  Collective over
    the group (handle exchange).  Both caps 0 / None disables."""
    old = _XGMI.pop(id(group), None)
    if old is not None:
        old.close()
    ag = cap_bytes if gather_cap_bytes is None else gather_cap_bytes
    if cap_bytes or ag:
        from .xgmi import XgmiAllReduce  # noqa: PLC0415
        _XGMI[id(group)] = XgmiAllReduce(group, cap_bytes or 0, ag or 0, timeout_ms=timeout_ms)
    return _XGMI.get(id(group))


def fold_xgmi_error(t):
    """``t`` (a float tensor on the device, e.g. the local grad-norm square)
    turned to +inf where any registered one-shot collective has timed out, so
    the non-finite-norm skip drops the step on every rank after the norm's
    all-reduce, with no host sync (NaN-poisoned activations must
    never reach the weights)."""
    for xg in _XGMI.values():
        err = xg.error_tensor()
        if err is not None and err.device == t.device:
            t = torch.where(err.to(t.dtype) != 0, torch.full_like(t, float("inf")), t)
    return t


def check_xgmi():
    """Raise :class:`parallel.xgmi.XgmiError` if any registered one-shot
    collective timed out waiting for a peer (cheap: one 4-byte read per
    communicator; synchronises the device)."""
    for xg in _XGMI.values():
        xg.check()


def xgmi_allreduce_of(group):
    return _XGMI.get(id(group))


def loopback_size(group):
    return _LOOPBACK.get(id(group))


def name_group(group, name):
    """Give a process group a readable name in the accounting table."""
    _GROUP_NAMES[id(group)] = name
    try:
        _GROUP_SIZES[name] = _LOOPBACK.get(id(group)) or dist.get_world_size(group)
    except (RuntimeError, ValueError):
        pass


def group_size(name):
    """Ranks of the named group (None if unknown)."""
    return _GROUP_SIZES.get(name)


def _key(op, group):
    return f"{op}/{_GROUP_NAMES.get(id(group), 'world' if group is None else 'group')}"


def _account(key, nbytes):
    rec = _STATS.get(key)
    if rec is None:
        rec = _STATS[key] = [0, 0, 0.0]
    rec[0] += 1
    rec[1] += nbytes


def _events_on(t):
    # (no timing events inside a hipGraph capture: collectives of a captured
    # TP decode step, inference/hip_graph.py)
    return _TIMING[0] and t.is_cuda and not torch.cuda.is_current_stream_capturing()


def _add_ms(key, ms):
    rec = _STATS.get(key)
    if rec is None:  # e.g. "p2p/.." (bytes are accounted per direction)
        rec = _STATS[key] = [0, 0, 0.0]
    rec[2] += ms


def _fold_events(block=False):
    keep = []
    for key, s, e in _PENDING_EVENTS:
        if block or e.query():
            _add_ms(key, s.elapsed_time(e))
        else:
            keep.append((key, s, e))
    _PENDING_EVENTS[:] = keep


def report(reset=True):
    """{key: (count, bytes, ms)} since the last report.  Also raises if a
    one-shot xGMI collective timed out waiting for a peer since it was set up
    (its results would be wrong: parallel/xgmi.py)."""
    _fold_events(block=True)
    for xg in _XGMI.values():
        xg.check()
    out = {k: tuple(v) for k, v in _STATS.items()}
    if reset:
        _STATS.clear()
    return out


def format_report(rep):
    parts = []
    for k, (n, b, ms) in rep.items():
        s = f"{k}: {n}x {b / 2**20:.1f} MiB"
        if ms > 0:
            s += f" {ms:.1f} ms ({b / 2**30 / max(ms, 1e-6) * 1e3:.1f} GiB/s)"
        parts.append(s)
    return " | ".join(parts)


_INT_OF = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}


def _bitwise_equal(a, b):
    """Equality that treats NaN payloads as values (a NaN grad is not a race)."""
    if a.is_floating_point():
        it = _INT_OF[a.element_size()]
        return torch.equal(a.contiguous().view(it), b.contiguous().view(it))
    return torch.equal(a, b)


class Work:
    """Handle of an issued collective (``wait()`` makes the result visible to
    the current stream)."""

    __slots__ = ("_work", "_run", "_key", "_start", "_done", "_snap", "_watch", "_t0")

    def __init__(self, work=None, run=None, key=None, start=None, watch=None, snap=None,
                 t0=None):
        self._work, self._run, self._key, self._start = work, run, key, start
        self._watch, self._snap = watch, snap
        self._t0 = t0  # host clock at issue (timing of host-side collectives: gloo)
        self._done = False

    def wait(self):
        if self._done:
            return
        self._done = True
        if self._run is not None:  # race-check mode: verify, then run for real
            watch = self._watch.detach() if isinstance(self._watch, _SendWatch) else self._watch
            if not _bitwise_equal(watch, self._snap):
                raise CommRaceError(
                    f"{self._key}: buffer written while the collective was in flight "
                    f"(between launch and wait)")
            r = self._run()
            if r is not None and hasattr(r, "wait"):
                r.wait()  # stream-ordered work (loopback stream, p2p requests)
        elif self._work is not None:
            self._work.wait()
        if self._start is not None:
            end = torch.cuda.Event(enable_timing=True)
            end.record()
            _PENDING_EVENTS.append((self._key, self._start, end))
        elif self._t0 is not None:
            _add_ms(self._key, (time.perf_counter() - self._t0) * 1e3)


class _StreamWork:
    """Handle of loopback work queued on the loopback stream (the stand-in for
    RCCL's own stream): ``wait()`` orders the current stream behind it."""

    __slots__ = ("_ev",)

    def __init__(self, ev):
        self._ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self._ev)


_LOOP_STREAMS = {}
# EMA_LOOPBACK_STREAM=1: loopback copies on a stream of their own, as RCCL's
# kernels run.  Off by default: the copies are CU kernels (RCCL's run on a few
# CUs), and beside the persistent GEMMs they cost both TP proxies 4 %
# (profiles/r5x_loopback_stream_ab.txt).
_LOOP_SIDE_STREAM = os.environ.get("EMA_LOOPBACK_STREAM", "0") == "1"
# Simulated peers' slots of a loopback all-gather into a persistent scratch
# buffer (parallel/buffers.py) are written once per (buffer, generation,
# range): between two hand-outs of the buffer with the same view nothing else
# writes it, so the slots still hold the finite activations written then, and
# the per-call traffic is this rank's own slot, as the proxy's compute-only
# accounting assumes.  A new generation (the buffer re-allocated, or handed out
# with another shape, i.e. possibly written by another user) refills them.
# Any other output (a fresh allocation that may hold recycled bytes) is fully
# written each call.  Proxy-only: a real all-gather writes every slot anyway.
_LOOP_FILLED = set()  # (buffer key, generation, storage offset, numel)


def _loop_async(fn, tensors):
    """Run a loopback collective's copies the way RCCL runs a collective: on a
    stream of its own that first waits for the work already queued on the
    current stream, overlapping whatever the caller queues next."""
    if not tensors[0].is_cuda or not _LOOP_SIDE_STREAM:
        fn()
        return None
    cur = torch.cuda.current_stream()
    s = _LOOP_STREAMS.get(cur.device)
    if s is None:
        s = _LOOP_STREAMS[cur.device] = torch.cuda.Stream(device=cur.device)
    s.wait_stream(cur)
    with torch.cuda.stream(s):
        fn()
    for t in tensors:
        t.record_stream(s)
    ev = torch.cuda.Event()
    ev.record(s)
    return _StreamWork(ev)


def _host_t0(t):
    return time.perf_counter() if _TIMING[0] and not t.is_cuda else None


def _issue(op, group, tensor_for_bytes, watch, fn, async_op):
    key = _key(op, group)
    nbytes = tensor_for_bytes.numel() * tensor_for_bytes.element_size()
    _account(key, nbytes)
    if _trace.tracing():
        with _trace.trace_range(f"comm:{key} {nbytes / 2**20:.1f}MiB"):
            return _issue_inner(key, tensor_for_bytes, watch, fn, async_op)
    return _issue_inner(key, tensor_for_bytes, watch, fn, async_op)


def _issue_inner(key, tensor_for_bytes, watch, fn, async_op):
    start = None
    if _events_on(tensor_for_bytes):
        start = torch.cuda.Event(enable_timing=True)
        start.record()
    t0 = _host_t0(tensor_for_bytes)
    if async_op and _CHECK:
        return Work(run=lambda: fn(False), key=key, start=start, watch=watch,
                    snap=watch.detach().clone(), t0=t0)
    w = fn(async_op)
    h = Work(work=w, key=key, start=start, t0=t0)
    if not async_op:
        h.wait()
        return None
    return h


def _op(op):
    if op == "avg":
        return dist.ReduceOp.AVG
    if op == "sum" or op is None:
        return dist.ReduceOp.SUM
    if op == "max":
        return dist.ReduceOp.MAX
    return op


def all_reduce(tensor, group=None, async_op=False, op="sum"):
    """In-place all-reduce; ``op='avg'`` averages inside the collective (ncclAvg)."""
    rop = _op(op)
    if id(group) in _LOOPBACK:
        return _issue("all_reduce", group, tensor, tensor, lambda a: None, async_op)
    xg = _XGMI.get(id(group))
    if xg is not None and rop == dist.ReduceOp.SUM and xg.eligible(tensor):
        # stream-ordered kernel: complete for the current stream when issued
        def oneshot(a):
            xg(tensor)
        return _issue("all_reduce_xgmi", group, tensor, tensor, oneshot, async_op)
    return _issue("all_reduce", group, tensor, tensor,
                  lambda a: dist.all_reduce(tensor, op=rop, group=group, async_op=a), async_op)


def reduce_scatter_into(output, inp, group=None, async_op=False, op="sum"):
    """``output`` = this rank's dim-0 chunk of the reduction of ``inp`` over ranks.
    ``output`` may alias the matching chunk of ``inp`` (in-place form)."""
    rop = _op(op)
    src = inp if inp.is_contiguous() else inp.contiguous()
    n = _LOOPBACK.get(id(group))
    if n:
        def loop(a):
            own = src.view(n, *output.shape)[0]
            if output.data_ptr() != own.data_ptr():
                return _loop_async(lambda: output.copy_(own), [output, src])
            return None
        return _issue("reduce_scatter", group, src, src, loop, async_op)
    return _issue("reduce_scatter", group, src, src,
                  lambda a: dist.reduce_scatter_tensor(output, src, op=rop, group=group,
                                                       async_op=a), async_op)


def all_gather_into(output, inp, group=None, async_op=False):
    """``output`` = concat over ranks of ``inp`` along dim 0.  ``inp`` may alias
    this rank's chunk of ``output`` (in-place form)."""
    src = inp if inp.is_contiguous() else inp.contiguous()
    n = _LOOPBACK.get(id(group))
    if n:
        def loop(a):
            # every simulated peer's slot gets this rank's shard: the output is
            # fully written each call (as a real all-gather writes it), so no
            # stale / non-finite bytes of a recycled allocation reach the loss
            # (ADVICE r4); the copies run on the loopback stream, overlapping
            # compute as RCCL's would, with a real rank's write traffic
            rows = output.view(n, -1)
            flat = src.reshape(1, -1)
            from .buffers import get_global_memory_buffer  # noqa: PLC0415
            owner = get_global_memory_buffer().owner(output)
            key = None if owner is None else owner + (output.storage_offset(), output.numel())
            peers = key is None or key not in _LOOP_FILLED

            def fill():
                if rows[0].data_ptr() != src.data_ptr():
                    rows[0:1].copy_(flat)
                if peers:
                    rows[1:].copy_(flat.expand(n - 1, -1))
            if key is not None:
                _LOOP_FILLED.add(key)
            return _loop_async(fill, [output, src])
        return _issue("all_gather", group, output, src, loop, async_op)
    xg = _XGMI.get(id(group))
    if xg is not None and xg.gather_eligible(output, src):
        def oneshot(a):
            xg.all_gather(output, src)
        return _issue("all_gather_xgmi", group, output, src, oneshot, async_op)
    return _issue("all_gather", group, output, src,
                  lambda a: dist.all_gather_into_tensor(output, src, group=group, async_op=a),
                  async_op)


def broadcast(tensor, src, group=None, async_op=False):
    if id(group) in _LOOPBACK:
        return _issue("broadcast", group, tensor, tensor, lambda a: None, async_op)
    return _issue("broadcast", group, tensor, tensor,
                  lambda a: dist.broadcast(tensor, src=src, group=group, async_op=a), async_op)


def p2p(ops, group=None, async_op=False):
    """Batched point-to-point exchange: ``ops`` = [(kind, tensor, peer)] with
    kind ``"send"`` / ``"recv"`` and ``peer`` a global rank; posted in list
    order as one ``batch_isend_irecv`` group (RCCL / NCCL match a peer pair's
    messages in posting order).  Returns a ``Work`` when ``async_op``."""
    ops = [o for o in ops if o is not None]
    if not ops:
        return None
    sent = [t for k, t, _ in ops if k == "send"]
    recvd = [t for k, t, _ in ops if k == "recv"]
    for kind, ts in (("p2p_send", sent), ("p2p_recv", recvd)):
        if ts:
            _account(_key(kind, group), sum(t.numel() * t.element_size() for t in ts))

    def fn(a):
        reqs = dist.batch_isend_irecv(
            [dist.P2POp(dist.isend if k == "send" else dist.irecv, t, peer, group)
             for k, t, peer in ops])
        if not a:
            for r in reqs:
                r.wait()
            return None
        return _Reqs(reqs)

    ref = (sent or recvd)[0]
    key = _key("p2p", group)
    if _trace.tracing():
        with _trace.trace_range(f"comm:{key}"):
            return _p2p_issue(key, ref, sent, fn, async_op)
    return _p2p_issue(key, ref, sent, fn, async_op)


class _Reqs:
    __slots__ = ("reqs",)

    def __init__(self, reqs):
        self.reqs = reqs

    def wait(self):
        for r in self.reqs:
            r.wait()


def _p2p_issue(key, ref, sent, fn, async_op):
    start = None
    if _events_on(ref):
        start = torch.cuda.Event(enable_timing=True)
        start.record()
    t0 = _host_t0(ref)
    if async_op and _CHECK and sent:
        # Only pure sends are deferred (a receive must complete before its
        # consumer runs): snapshot the send buffers, verify and send at wait().
        watch = torch.cat([t.detach().reshape(-1).view(torch.uint8) for t in sent]) \
            if len(sent) > 1 else sent[0].detach().reshape(-1).view(torch.uint8)
        return Work(run=lambda: fn(False), key=key, start=start, watch=_SendWatch(sent),
                    snap=watch.clone(), t0=t0)
    w = fn(async_op)
    h = Work(work=w, key=key, start=start, t0=t0)
    if not async_op:
        h.wait()
        return None
    return h


class _SendWatch:
    """The concatenated bytes of the send buffers, for the race check."""

    def __init__(self, tensors):
        self.tensors = tensors

    def detach(self):
        ts = [t.detach().reshape(-1).view(torch.uint8) for t in self.tensors]
        return torch.cat(ts) if len(ts) > 1 else ts[0]

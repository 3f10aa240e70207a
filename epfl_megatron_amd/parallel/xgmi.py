"""One-shot all-reduce / all-gather over xGMI peer memory (``csrc/xgmi_allreduce.hip``).

SURVEY §5.8 ("a custom one-shot all-reduce / all-gather kernel over xGMI peer
memory (IPC handles) for small, latency-bound messages ... RCCL stays the
default and the fallback").  The reference has no equivalent: every TP
all-reduce goes to NCCL (``megatron/core/tensor_parallel/mappings.py:15-26``).

The messages this targets are the TP all-reduces of a decode step: two per
layer of ``[b, h]`` (8 KiB at batch 1 on a 4096-wide model).  A ring all-reduce
moves such a message through 2(W-1) dependent link hops plus RCCL's launch and
proxy handshakes; the one-shot form is one kernel: every rank writes its
message into a slot of every peer's IPC-mapped buffer (W-1 concurrent xGMI
writes over W-1 different point-to-point links), raises a flag per 4 KiB chunk,
and sums the W slots from its own HBM once the peers' flags are up.  The bytes
each link carries are the message once, against 2(W-1)/W messages of a ring
spread over fewer links, and there is no second phase.

Use: ``comm.enable_xgmi_allreduce(group, cap_bytes)`` (``--tp_xgmi_allreduce_kb``
does it for the TP group at initialisation); ``comm.all_reduce`` then routes
sum all-reduces of contiguous bf16 / fp16 / fp32 CUDA tensors of at most
``cap_bytes`` (16-byte sized and aligned) on that group here, everything else
to RCCL, and ``comm.all_gather_into`` likewise the all-gathers whose
per-rank message fits (e.g. the vocab-parallel decode logits).  Capturable in
a hipGraph (epochs live on the device).

Routing is decided from rank-uniform properties only (dtype, element count,
contiguity): a rank whose tensor happens to be misaligned stages it through
an aligned buffer instead of taking RCCL while its peers take the kernel (which
would hang or time out).  All-reduces and all-gathers have separate caps
(``--tp_xgmi_allreduce_kb`` / ``--tp_xgmi_allgather_kb``): the all-gather cap
covers the multi-MiB sequence-parallel ``[s/tp, b, h]`` pieces.

A wait on a peer is bounded by wall clock: ``timeout_ms`` per communicator
(default 60 s, or ``EMA_XGMI_TIMEOUT_MS``; ``--tp_xgmi_timeout_ms`` in
training).  The bound is long on purpose: TP ranks drift apart through host
work (checkpoint writes, first-iteration setup, a GC pause), and a late but
healthy peer must not trip it; a latency-critical caller (decode serving) can
pass a short one.  A dead peer ends the kernel with NaN-filled output and the
device error word set.  The optimizer folds that word into the grad-norm
reduction (:meth:`error_tensor`, ``comm.fold_xgmi_error``): every rank then
skips the step on device, with no host sync; :meth:`check` (every training log
line, the start of ``save_checkpoint``, after every generate call) raises.

Verified on one MI355X with 2 and 4 processes sharing the GPU
(``tests/test_xgmi_gpu.py``: same-device IPC mappings; the flag / parity
protocol and the kernel are the ones a multi-GPU run executes, the transport
there is xGMI instead of local HBM).  Not yet measured on an 8-GPU node, so
it is opt-in.
"""
import torch
import torch.distributed as dist


def _ext():
    from ..ops._ext import ext  # noqa: PLC0415  (raises when the extension is missing)
    return ext()


class XgmiError(RuntimeError):
    pass


class XgmiAllReduce:
    """One registered one-shot all-reduce communicator over ``group`` (2..8
    ranks, one GPU each; ranks sharing a GPU also work, as in the tests)."""

    DTYPES = (torch.bfloat16, torch.float16, torch.float32)

    def __init__(self, group=None, cap_bytes=1 << 20, gather_cap_bytes=None, timeout_ms=None):
        ar = int(cap_bytes)
        ag = ar if gather_cap_bytes is None else int(gather_cap_bytes)
        cap = max(ar, ag)
        if cap <= 0 or ar % 4096 or ag % 4096 or ar < 0 or ag < 0:
            raise ValueError("caps must be non-negative multiples of 4096 (one positive)")
        self.ar_cap, self.ag_cap = ar, ag
        self._stage = {}
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if not 2 <= self.world <= 8:
            raise ValueError("xGMI one-shot all-reduce needs 2..8 ranks")
        self.cap = cap
        C = _ext()
        self.id, handle = C.xgmi_create(self.rank, self.world, cap)
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(handle.numpy().tobytes()), group=group)
        table = torch.frombuffer(bytearray(b"".join(handles)), dtype=torch.uint8)
        C.xgmi_open(self.id, table.view(self.world, -1))
        if timeout_ms is not None:
            C.xgmi_set_timeout(self.id, int(timeout_ms))
        self.timeout_ms = C.xgmi_get_timeout(self.id)
        self._err = C.xgmi_error_tensor(self.id)
        dist.barrier(group=group)

    def _fits(self, t, cap):
        # rank-uniform: dtype, size and contiguity agree across the TP group
        # (never the address, which can differ per rank: ADVICE r4)
        nbytes = t.numel() * t.element_size()
        return (t.is_cuda and t.dtype in self.DTYPES and t.is_contiguous() and 0 < nbytes <= cap
                and nbytes % 16 == 0)

    def eligible(self, t):
        return self._fits(t, self.ar_cap)

    def _aligned(self, t, key):
        """``t`` itself when 16-B aligned, else a cached aligned staging copy."""
        if t.data_ptr() % 16 == 0:
            return t, False
        buf = self._stage.get(key)
        if buf is None or buf.numel() != t.numel() or buf.dtype != t.dtype or buf.device != t.device:
            buf = torch.empty_like(t, memory_format=torch.contiguous_format)
            self._stage[key] = buf
        buf.copy_(t)
        return buf, True

    def __call__(self, t, out=None):
        """``out`` (default: ``t``, in place) = sum of ``t`` over the group, on
        the current stream."""
        dst = t if out is None else out
        src, _ = self._aligned(t, "ar_in")
        if out is None or out.data_ptr() % 16:
            o = src if out is None else self._aligned(out, "ar_out")[0]
        else:
            o = out
        _ext().xgmi_all_reduce(self.id, src, o)
        if o.data_ptr() != dst.data_ptr():
            dst.copy_(o)
        return dst

    def gather_eligible(self, out, inp):
        return (self._fits(inp, self.ag_cap) and out.is_cuda and out.dtype == inp.dtype
                and out.is_contiguous() and out.numel() == self.world * inp.numel())

    def all_gather(self, out, inp):
        """``out`` = concat over ranks of ``inp`` along dim 0 (``inp`` may be
        this rank's chunk of ``out``), on the current stream."""
        src, _ = self._aligned(inp, "ag_in")
        o, staged = self._aligned(out, "ag_out") if out.data_ptr() % 16 else (out, False)
        _ext().xgmi_all_gather(self.id, src, o, self.world)
        if staged:
            out.copy_(o)
        return out

    def error_tensor(self):
        """Device int32 [1]: nonzero once a peer wait has timed out."""
        return self._err

    def check(self):
        """Raise if a wait timed out (a peer never arrived); synchronises."""
        if _ext().xgmi_error(self.id):
            raise XgmiError("xGMI one-shot all-reduce: a peer did not arrive within the wait "
                            "bound; results since then are invalid")

    def close(self):
        self._err = None
        if self.id is not None:
            _ext().xgmi_destroy(self.id)
            self.id = None

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

    def __init__(self, group=None, cap_bytes=1 << 20):
        cap = int(cap_bytes)
        if cap <= 0 or cap % 4096:
            raise ValueError("cap_bytes must be a positive multiple of 4096")
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
        dist.barrier(group=group)

    def eligible(self, t):
        nbytes = t.numel() * t.element_size()
        return (t.is_cuda and t.dtype in self.DTYPES and t.is_contiguous() and 0 < nbytes <= self.cap
                and nbytes % 16 == 0 and t.data_ptr() % 16 == 0)

    def __call__(self, t, out=None):
        """``out`` (default: ``t``, in place) = sum of ``t`` over the group, on
        the current stream."""
        _ext().xgmi_all_reduce(self.id, t, t if out is None else out)
        return t if out is None else out

    def gather_eligible(self, out, inp):
        return (self.eligible(inp) and out.is_cuda and out.dtype == inp.dtype and out.is_contiguous()
                and out.numel() == self.world * inp.numel() and out.data_ptr() % 16 == 0)

    def all_gather(self, out, inp):
        """``out`` = concat over ranks of ``inp`` along dim 0 (``inp`` may be
        this rank's chunk of ``out``), on the current stream."""
        _ext().xgmi_all_gather(self.id, inp, out, self.world)
        return out

    def check(self):
        """Raise if a wait timed out (a peer never arrived); synchronises."""
        if _ext().xgmi_error(self.id):
            raise XgmiError("xGMI one-shot all-reduce: a peer did not arrive within the wait "
                            "bound; results since then are invalid")

    def close(self):
        if self.id is not None:
            _ext().xgmi_destroy(self.id)
            self.id = None

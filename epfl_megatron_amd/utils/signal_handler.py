"""Graceful preemption: every rank learns that *some* rank got SIGTERM.

(reference ``megatron/dist_signal_handler.py``)  The flag is all-gathered each
iteration so all ranks checkpoint and exit at the same step.
"""
import signal

import torch
import torch.distributed as dist


def _gather_flags(flag):
    if not (dist.is_available() and dist.is_initialized()):
        return [flag]
    dev = torch.device("cuda", torch.cuda.current_device()) \
        if torch.cuda.is_available() and dist.get_backend() != "gloo" else torch.device("cpu")
    t = torch.tensor([int(flag)], dtype=torch.int32, device=dev)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [bool(x.item()) for x in out]


class DistributedSignalHandler:
    def __init__(self, sig=signal.SIGTERM):
        self.sig = sig
        self._received = False
        self._released = True
        self._original = None

    def signals_received(self):
        return _gather_flags(self._received)

    def __enter__(self):
        self._received = False
        self._released = False
        self._original = signal.getsignal(self.sig)

        def _handler(signum, frame):
            self._received = True

        signal.signal(self.sig, _handler)
        return self

    def __exit__(self, exc_type, exc, tb):
        self.release()

    def release(self):
        if self._released:
            return False
        signal.signal(self.sig, self._original)
        self._released = True
        return True

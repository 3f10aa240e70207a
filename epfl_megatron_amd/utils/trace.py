"""Named ranges for timeline profilers.

``trace_range(name)`` marks a region for BOTH consumers:

* ``roctx`` (``torch.cuda.nvtx`` is roctx on ROCm builds): shows as a marker
  range in ``rocprofv3 --marker-trace`` / rocprof-sys timelines next to the
  kernels it encloses;
* ``torch.profiler`` (``record_function``): shows in the PyTorch trace.

Off by default (zero overhead: a shared null context).  Enabled by
``--timing_log_level 2`` (``training.py``) or ``EMA_TRACE=1``.  Ranges are put
around every transformer layer (forward; the backward shows as the autograd
region of the same name), every micro-batch forward / backward of the
pipeline schedules, the optimizer phases, and every collective issued through
``parallel/comm.py`` (``comm:<op>/<group>`` with the byte count).
"""
import contextlib
import os

import torch

_ON = [os.environ.get("EMA_TRACE", "0") == "1"]
_NULL = contextlib.nullcontext()


def set_tracing(enabled):
    _ON[0] = bool(enabled)


def tracing():
    return _ON[0]


@contextlib.contextmanager
def _range(name):
    pushed = False
    try:
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
            pushed = True
    except Exception:  # pragma: no cover - roctx unavailable
        pushed = False
    with torch.autograd.profiler.record_function(name):
        try:
            yield
        finally:
            if pushed:
                torch.cuda.nvtx.range_pop()


def trace_range(name):
    """Context manager; a no-op unless tracing is on."""
    return _range(name) if _ON[0] else _NULL

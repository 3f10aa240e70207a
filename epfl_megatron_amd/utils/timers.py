"""Levelled wall-clock timers (reference ``megatron/timers.py``).

Same names, levels (0/1/2) and min/max/all cross-rank report, but the GPU
timeline is measured with HIP events recorded on the current stream instead of
a ``torch.cuda.synchronize()`` in every start/stop: start/stop are
asynchronous; the events are only resolved when ``elapsed()`` is read at log
time.  ``barrier=True`` keeps the reference's optional cross-rank barrier.
"""
import time

import torch
import torch.distributed as dist


class _DummyTimer:
    def start(self, barrier=False):
        pass

    def stop(self, barrier=False):
        pass

    def reset(self):
        pass

    def elapsed(self, reset=True, barrier=False):
        raise Exception("dummy timer should not be used to calculate elapsed time")


class Timer:
    def __init__(self, name):
        self.name = name
        self._use_events = torch.cuda.is_available()
        self._pairs = []          # recorded (start_event, stop_event)
        self._host_elapsed = 0.0  # CPU path accumulation
        self._started = False
        self._cur = None
        self._t0 = 0.0
        self._barrier_group = None

    def set_barrier_group(self, group):
        self._barrier_group = group

    def _barrier(self, barrier):
        if barrier and dist.is_initialized():
            dist.barrier(group=self._barrier_group)

    def start(self, barrier=False):
        if self._started:
            raise AssertionError(f"timer {self.name} has already been started")
        self._barrier(barrier)
        if self._use_events:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._cur = ev
        else:
            self._t0 = time.time()
        self._started = True

    def stop(self, barrier=False):
        if not self._started:
            raise AssertionError(f"timer {self.name} is not started")
        self._barrier(barrier)
        if self._use_events:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._pairs.append((self._cur, ev))
            self._cur = None
        else:
            self._host_elapsed += time.time() - self._t0
        self._started = False

    def reset(self):
        self._pairs = []
        self._host_elapsed = 0.0
        self._started = False
        self._cur = None

    def _resolve(self):
        total = self._host_elapsed
        for s, e in self._pairs:
            e.synchronize()
            total += s.elapsed_time(e) / 1000.0
        return total

    def elapsed(self, reset=True, barrier=False):
        was_started = self._started
        if was_started:
            self.stop(barrier=barrier)
        total = self._resolve()
        if reset:
            self.reset()
        else:
            self._host_elapsed = total
            self._pairs = []
        if was_started:
            self.start(barrier=barrier)
        return total


class Timers:
    """Group of named timers with a log level filter."""

    def __init__(self, log_level, log_option):
        self._log_level = log_level
        self._log_option = log_option
        self._timers = {}
        self._levels = {}
        self._dummy = _DummyTimer()
        self._max_level = 2

    def __call__(self, name, log_level=None):
        if name in self._timers:
            if log_level is not None and log_level != self._levels[name]:
                raise AssertionError(f"input log level {log_level} does not match already "
                                     f"existing log level {self._levels[name]} for {name} timer")
            return self._timers[name]
        if log_level is None:
            log_level = self._max_level
        if log_level > self._max_level:
            raise AssertionError(f"log level {log_level} is larger than max supported log "
                                 f"level {self._max_level}")
        if log_level > self._log_level:
            return self._dummy
        self._timers[name] = Timer(name)
        self._levels[name] = log_level
        return self._timers[name]

    def _gather_elapsed(self, names, reset, barrier):
        if barrier and dist.is_initialized():
            dist.barrier()
        world = dist.get_world_size() if dist.is_initialized() else 1
        rank = dist.get_rank() if dist.is_initialized() else 0
        values = torch.zeros(len(names), dtype=torch.float)
        for i, n in enumerate(names):
            if n in self._timers:
                values[i] = self._timers[n].elapsed(reset=reset)
        if world == 1:
            return values.view(1, -1)
        dev = torch.device("cuda", torch.cuda.current_device()) \
            if torch.cuda.is_available() and dist.get_backend() != "gloo" else torch.device("cpu")
        local = values.to(dev)
        out = [torch.zeros_like(local) for _ in range(world)]
        dist.all_gather(out, local)
        return torch.stack(out).cpu()

    def _min_max(self, names, reset, barrier):
        allv = self._gather_elapsed(names, reset, barrier)
        res = {}
        for i, n in enumerate(names):
            col = allv[:, i]
            col = col[col > 0.0]
            if col.numel() > 0:
                res[n] = (col.min().item() * 1000.0, col.max().item() * 1000.0)
        return res

    def _string(self, names, normalizer, reset, barrier):
        if normalizer <= 0.0:
            raise AssertionError("normalizer should be positive")
        if self._log_option in ("max", "minmax"):
            mm = self._min_max(names, reset, barrier)
            if not mm:
                return None
            head = "(min, max) time across ranks (ms):" if self._log_option == "minmax" \
                else "max time across ranks (ms):"
            s = head
            for n, (lo, hi) in mm.items():
                if self._log_option == "minmax":
                    s += f"\n    {n + ' ':.<48}: ({lo / normalizer:.2f}, {hi / normalizer:.2f})"
                else:
                    s += f"\n    {n + ' ':.<48}: {hi / normalizer:.2f}"
            return s
        allv = self._gather_elapsed(names, reset, barrier)
        s = "times across ranks (ms):"
        for i, n in enumerate(names):
            s += f"\n  {n}:"
            for r in range(allv.shape[0]):
                if allv[r, i] > 0:
                    s += f"\n     rank {r:2d}: {allv[r, i] * 1000.0 / normalizer:.2f}"
        return s

    def log(self, names, rank=None, normalizer=1.0, reset=True, barrier=False):
        s = self._string(names, normalizer, reset, barrier)
        if rank is None:
            rank = (dist.get_world_size() - 1) if dist.is_initialized() else 0
        me = dist.get_rank() if dist.is_initialized() else 0
        if me == rank and s is not None:
            print(s, flush=True)

    def write(self, names, writer, iteration, normalizer=1.0, reset=False, barrier=False):
        if normalizer <= 0.0:
            raise AssertionError("normalizer should be positive")
        mm = self._min_max(names, reset, barrier)
        if writer is not None:
            for n, (_, hi) in mm.items():
                writer.add_scalar(n + "-time", hi / normalizer, iteration)

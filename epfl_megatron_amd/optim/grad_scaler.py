"""Loss scalers for fp16 (reference ``megatron/optimizer/grad_scaler.py``).

``update(found_inf)`` accepts a device bool/float tensor: the dynamic scaler
keeps its growth / hysteresis trackers on the device and updates them with
``torch.where`` so the optimizer step never waits for the GPU.  The checkpoint
format (python ints for the trackers) is unchanged."""
import torch


class MegatronGradScaler:
    def __init__(self, initial_scale):
        if initial_scale <= 0.0:
            raise AssertionError("initial scale must be positive")
        dev = torch.cuda.current_device() if torch.cuda.is_available() else "cpu"
        self._scale = torch.tensor([initial_scale], dtype=torch.float, device=dev)

    @property
    def scale(self):
        return self._scale

    @property
    def inv_scale(self):
        return self._scale.double().reciprocal().float()

    def update(self, found_inf):
        raise NotImplementedError

    def state_dict(self):
        raise NotImplementedError

    def load_state_dict(self, state_dict):
        raise NotImplementedError


class ConstantGradScaler(MegatronGradScaler):
    def update(self, found_inf):
        pass

    def state_dict(self):
        return {}

    def load_state_dict(self, state_dict):
        pass


class DynamicGradScaler(MegatronGradScaler):
    """Halve on overflow after ``hysteresis`` consecutive infs; double after
    ``growth_interval`` clean steps; never below ``min_scale``."""

    def __init__(self, initial_scale, min_scale, growth_factor, backoff_factor, growth_interval,
                 hysteresis):
        super().__init__(initial_scale)
        if not (0.0 < min_scale <= initial_scale):
            raise AssertionError("invalid min scale")
        if growth_factor <= 1.0 or not (0.0 < backoff_factor < 1.0):
            raise AssertionError("invalid growth/backoff factors")
        if growth_interval <= 0 or hysteresis <= 0:
            raise AssertionError("invalid growth interval / hysteresis")
        dev = self._scale.device
        self.min_scale = torch.tensor([min_scale], dtype=torch.float, device=dev)
        self.growth_factor = torch.tensor([growth_factor], dtype=torch.float, device=dev)
        self.backoff_factor = torch.tensor([backoff_factor], dtype=torch.float, device=dev)
        self.growth_interval = growth_interval
        self.hysteresis = hysteresis
        self._growth = torch.zeros(1, dtype=torch.int32, device=dev)
        self._hyst = torch.full((1,), hysteresis, dtype=torch.int32, device=dev)

    def update(self, found_inf):
        dev = self._scale.device
        found = torch.as_tensor(found_inf, device=dev).reshape(1).bool()
        zero = torch.zeros_like(self._growth)
        growth = torch.where(found, zero, self._growth + 1)
        hyst = torch.where(found, self._hyst - 1, self._hyst)
        backoff = found & (hyst <= 0)
        scale = torch.where(backoff, torch.max(self._scale * self.backoff_factor, self.min_scale),
                            self._scale)
        grow = (~found) & (growth == self.growth_interval)
        self._growth = torch.where(grow, zero, growth)
        self._hyst = torch.where(grow, torch.full_like(hyst, self.hysteresis), hyst)
        self._scale = torch.where(grow, scale * self.growth_factor, scale)

    @property
    def _growth_tracker(self):
        return int(self._growth.item())

    @property
    def _hysteresis_tracker(self):
        return int(self._hyst.item())

    def state_dict(self):
        return {"scale": self._scale, "growth_tracker": self._growth_tracker,
                "hysteresis_tracker": self._hysteresis_tracker}

    def load_state_dict(self, sd):
        dev = self._scale.device
        self._scale = sd["scale"].to(dev)
        self._growth.fill_(int(sd["growth_tracker"]))
        self._hyst.fill_(int(sd["hysteresis_tracker"]))

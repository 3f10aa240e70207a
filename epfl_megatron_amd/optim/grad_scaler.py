"""Loss scalers for fp16 (reference ``megatron/optimizer/grad_scaler.py``)."""
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
        self._growth_tracker = 0
        self._hysteresis_tracker = hysteresis

    def update(self, found_inf):
        if found_inf:
            self._growth_tracker = 0
            self._hysteresis_tracker -= 1
            if self._hysteresis_tracker <= 0:
                self._scale = torch.max(self._scale * self.backoff_factor, self.min_scale)
        else:
            self._growth_tracker += 1
            if self._growth_tracker == self.growth_interval:
                self._growth_tracker = 0
                self._hysteresis_tracker = self.hysteresis
                self._scale = self._scale * self.growth_factor

    def state_dict(self):
        return {"scale": self._scale, "growth_tracker": self._growth_tracker,
                "hysteresis_tracker": self._hysteresis_tracker}

    def load_state_dict(self, sd):
        dev = self._scale.device
        self._scale = sd["scale"].to(dev)
        self._growth_tracker = sd["growth_tracker"]
        self._hysteresis_tracker = sd["hysteresis_tracker"]

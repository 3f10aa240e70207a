"""Class definitions that very old Megatron checkpoints pickled their loss
scalers as (``fp16.loss_scaler`` / ``megatron.fp16.loss_scaler``; reference
``megatron/fp16_deprecated/loss_scaler.py``, ``megatron/checkpointing.py:457-468``).

They only need to exist so such a checkpoint deserialises; the checkpoint
loader allow-lists them for ``torch.load(weights_only=True)`` under those
legacy module names (nothing in them executes on load: the unpickler only
restores attributes).
"""


class LossScaler:
    def __init__(self, scale=1):
        self.cur_scale = scale


class DynamicLossScaler:
    def __init__(self, init_scale=2 ** 32, scale_factor=2.0, scale_window=1000, min_scale=1,
                 delayed_shift=1, consecutive_hysteresis=False):
        self.cur_scale = init_scale
        self.cur_iter = 0
        self.last_overflow_iter = -1
        self.scale_factor = scale_factor
        self.scale_window = scale_window
        self.min_scale = min_scale
        self.delayed_shift = delayed_shift
        self.cur_hysteresis = delayed_shift
        self.consecutive_hysteresis = consecutive_hysteresis

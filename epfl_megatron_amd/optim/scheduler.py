"""LR / weight-decay schedule counted in samples
(reference ``megatron/optimizer_param_scheduler.py``)."""
import math


class OptimizerParamScheduler:
    def __init__(self, optimizer, max_lr, min_lr, lr_warmup_steps, lr_decay_steps, lr_decay_style,
                 start_wd, end_wd, wd_incr_steps, wd_incr_style, use_checkpoint_opt_param_scheduler=True,
                 override_opt_param_scheduler=False):
        self.optimizer = optimizer
        self.max_lr = float(max_lr)
        self.min_lr = min_lr
        if not (0.0 <= self.min_lr <= self.max_lr):
            raise AssertionError("need 0 <= min_lr <= max_lr")
        self.lr_warmup_steps = lr_warmup_steps
        self.num_steps = 0
        self.lr_decay_steps = lr_decay_steps
        if lr_decay_steps <= 0 or lr_warmup_steps >= lr_decay_steps:
            raise AssertionError("need 0 <= warmup < decay steps")
        self.lr_decay_style = lr_decay_style
        self.start_wd, self.end_wd = start_wd, end_wd
        if not (0.0 <= start_wd <= end_wd):
            raise AssertionError("need 0 <= start_wd <= end_wd")
        self.wd_incr_steps = wd_incr_steps
        self.wd_incr_style = wd_incr_style
        self.override_opt_param_scheduler = override_opt_param_scheduler
        self.use_checkpoint_opt_param_scheduler = use_checkpoint_opt_param_scheduler
        if override_opt_param_scheduler and use_checkpoint_opt_param_scheduler:
            raise AssertionError("both override and use-checkpoint are set.")
        self.step(0)
        print(f"> learning rate decay style: {self.lr_decay_style}", flush=True)

    def get_wd(self):
        if self.num_steps > self.wd_incr_steps:
            return self.end_wd
        if self.wd_incr_style == "constant":
            return self.end_wd
        r = float(self.num_steps) / float(self.wd_incr_steps)
        if self.wd_incr_style == "linear":
            coeff = r
        elif self.wd_incr_style == "cosine":
            coeff = 0.5 * (math.cos(math.pi * (1 - r)) + 1.0)
        else:
            raise Exception(f"{self.wd_incr_style} weight decay increment style is not supported.")
        return self.start_wd + coeff * (self.end_wd - self.start_wd)

    def get_lr(self):
        if self.lr_warmup_steps > 0 and self.num_steps <= self.lr_warmup_steps:
            return self.max_lr * float(self.num_steps) / float(self.lr_warmup_steps)
        if self.lr_decay_style == "constant":
            return self.max_lr
        if self.num_steps > self.lr_decay_steps:
            return self.min_lr
        if self.lr_decay_style == "inverse-square-root":
            warm = max(self.lr_warmup_steps, 1)
            num = max(self.num_steps, 1)
            return max(self.min_lr, self.max_lr * warm ** 0.5 / (num ** 0.5))
        r = float(self.num_steps - self.lr_warmup_steps) / \
            float(self.lr_decay_steps - self.lr_warmup_steps)
        if self.lr_decay_style == "linear":
            coeff = 1.0 - r
        elif self.lr_decay_style == "cosine":
            coeff = 0.5 * (math.cos(math.pi * r) + 1.0)
        else:
            raise Exception(f"{self.lr_decay_style} decay style is not supported.")
        return self.min_lr + coeff * (self.max_lr - self.min_lr)

    def step(self, increment):
        self.num_steps += increment
        lr = self.get_lr()
        wd = self.get_wd()
        for g in self.optimizer.param_groups:
            g["lr"] = lr * g.get("lr_mult", 1.0)
            g["weight_decay"] = wd * g.get("wd_mult", 1.0)

    def rollback(self, increment):
        """Undo ``step(increment)`` (the optimizer found the step skipped only
        after the fact — its non-finite check runs on the device)."""
        self.step(-increment)

    def state_dict(self):
        return {"max_lr": self.max_lr, "lr_warmup_steps": self.lr_warmup_steps,
                "num_steps": self.num_steps, "lr_decay_style": self.lr_decay_style,
                "lr_decay_steps": self.lr_decay_steps, "min_lr": self.min_lr,
                "start_wd": self.start_wd, "end_wd": self.end_wd,
                "wd_incr_style": self.wd_incr_style, "wd_incr_steps": self.wd_incr_steps}

    def _check_and_set(self, cls_value, sd_value, name):
        if self.override_opt_param_scheduler:
            print(f" > overriding {name} value to {cls_value}", flush=True)
            return cls_value
        if not self.use_checkpoint_opt_param_scheduler and cls_value != sd_value:
            raise AssertionError(f"OptimizerParamScheduler: class input value {cls_value} and "
                                 f"checkpoint value {sd_value} for {name} do not match")
        print(f" > using checkpoint value {sd_value} for {name}", flush=True)
        return sd_value

    def load_state_dict(self, sd):
        max_lr = sd.get("start_lr", sd.get("max_lr"))
        self.max_lr = self._check_and_set(self.max_lr, max_lr, "learning rate")
        self.min_lr = self._check_and_set(self.min_lr, sd["min_lr"], "minimum learning rate")
        warm = sd.get("warmup_iter", sd.get("warmup_steps", sd.get("lr_warmup_steps")))
        self.lr_warmup_steps = self._check_and_set(self.lr_warmup_steps, warm, "warmup iterations")
        decay = sd.get("end_iter", sd.get("decay_steps", sd.get("lr_decay_steps")))
        self.lr_decay_steps = self._check_and_set(self.lr_decay_steps, decay,
                                                  "total number of iterations")
        style = sd.get("decay_style", sd.get("lr_decay_style"))
        self.lr_decay_style = self._check_and_set(self.lr_decay_style, style,
                                                  "learning rate decay style")
        num_steps = sd.get("num_iters", sd.get("num_steps"))
        self.step(increment=num_steps)
        if "start_wd" in sd:
            self.start_wd = self._check_and_set(self.start_wd, sd["start_wd"], "start weight decay")
            self.end_wd = self._check_and_set(self.end_wd, sd["end_wd"], "end weight decay")
            self.wd_incr_steps = self._check_and_set(self.wd_incr_steps, sd["wd_incr_steps"],
                                                     "total number of weight decay iterations")
            self.wd_incr_style = self._check_and_set(self.wd_incr_style, sd["wd_incr_style"],
                                                     "weight decay incr style")

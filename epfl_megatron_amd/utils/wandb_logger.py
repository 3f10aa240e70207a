"""TensorBoard-compatible writer that also (optionally) logs to Weights & Biases.

Reference ``megatron/wandb_logger.py``: a ``SummaryWriter``-like shim on the
last rank; ``" vs "`` series (e.g. ``lm loss vs samples``) go to TensorBoard
only.  ``wandb`` is imported lazily; without it (or without network) the shim
keeps a local JSONL log so runs remain inspectable offline.
"""
import json
import os
import time
from dataclasses import dataclass, field
from typing import Optional


@dataclass
class WandBConfig:
    project: Optional[str] = None
    entity: Optional[str] = None
    run_id: Optional[str] = None
    resume: bool = False
    api_key: Optional[str] = None
    log_dir: Optional[str] = None
    config: dict = field(default_factory=dict)

    @staticmethod
    def from_args(args):
        return WandBConfig(project=args.wandb_project, entity=args.wandb_entity,
                           run_id=args.wandb_id, resume=args.wandb_resume,
                           api_key=args.wandb_api_key or os.environ.get("WANDB_API_KEY"),
                           log_dir=args.tensorboard_dir,
                           config={k: str(v) for k, v in vars(args).items()})


class WandbTBShim:
    def __init__(self, cfg: WandBConfig, tb_writer=None):
        self.cfg = cfg
        self.tb = tb_writer
        self._wandb = None
        self._pending = {}
        self._pending_step = None
        self._jsonl = None
        try:  # pragma: no cover - wandb is not installed in the CI image
            import wandb
            if cfg.api_key:
                os.environ["WANDB_API_KEY"] = cfg.api_key
            wandb.init(project=cfg.project, entity=cfg.entity, id=cfg.run_id,
                       resume="allow" if cfg.resume else None, config=cfg.config,
                       dir=cfg.log_dir)
            self._wandb = wandb
        except Exception:
            if cfg.log_dir:
                os.makedirs(cfg.log_dir, exist_ok=True)
                self._jsonl = open(os.path.join(cfg.log_dir, "metrics.jsonl"), "a")

    def add_scalar(self, name, value, step=None, **kw):
        if self.tb is not None:
            self.tb.add_scalar(name, value, step)
        if " vs " in name:
            return
        if self._pending_step is not None and step != self._pending_step:
            self.flush_all()
        self._pending_step = step
        self._pending[name] = float(value)

    def add_text(self, name, text, step=None):
        if self.tb is not None:
            self.tb.add_text(name, text, step)

    def flush_all(self):
        if not self._pending:
            return
        if self._wandb is not None:
            self._wandb.log(dict(self._pending), step=self._pending_step)
        elif self._jsonl is not None:
            rec = dict(self._pending, step=self._pending_step, time=time.time())
            self._jsonl.write(json.dumps(rec) + "\n")
            self._jsonl.flush()
        self._pending = {}

    def flush(self):
        self.flush_all()
        if self.tb is not None:
            self.tb.flush()

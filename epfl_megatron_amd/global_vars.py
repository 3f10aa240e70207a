"""Process-wide singletons (reference ``megatron/global_vars.py``)."""
import os
import sys

import torch

from .config.microbatches import build_num_microbatches_calculator
from .utils.timers import Timers

_G = {
    "args": None, "num_microbatches_calculator": None, "tokenizer": None,
    "tensorboard_writer": None, "adlr_autoresume": None, "timers": None,
    "signal_handler": None,
}


def _get(name, what=None):
    v = _G[name]
    if v is None and what is not None:
        raise AssertionError(f"{what} is not initialized.")
    return v


def get_args():
    return _get("args", "args")


def get_args_or_none():
    """The parsed args, or None outside an initialized run (library use)."""
    return _G["args"]


def get_num_microbatches():
    return _get("num_microbatches_calculator", "num microbatches calculator").get()


def get_current_global_batch_size():
    return _get("num_microbatches_calculator", "num microbatches calculator") \
        .get_current_global_batch_size()


def update_num_microbatches(consumed_samples, consistency_check=True):
    _get("num_microbatches_calculator", "num microbatches calculator") \
        .update(consumed_samples, consistency_check)


def get_tokenizer():
    return _get("tokenizer", "tokenizer")


def get_tensorboard_writer():
    return _G["tensorboard_writer"]


def get_adlr_autoresume():
    return _G["adlr_autoresume"]


def get_timers():
    return _get("timers", "timers")


def get_signal_handler():
    return _get("signal_handler", "signal handler")


def _set_signal_handler():
    from .utils.signal_handler import DistributedSignalHandler
    _G["signal_handler"] = DistributedSignalHandler().__enter__()


def set_global_variables(args, build_tokenizer=True):
    if args is None:
        raise AssertionError("args is None")
    _G["args"] = args
    _G["num_microbatches_calculator"] = build_num_microbatches_calculator(args)
    if build_tokenizer and getattr(args, "tokenizer_type", None) is not None:
        _build_tokenizer(args)
    _set_tensorboard_writer(args)
    _set_adlr_autoresume(args)
    _set_timers(args)
    if args.exit_signal_handler:
        _set_signal_handler()


def set_args(args):
    _G["args"] = args


def _build_tokenizer(args):
    from .tokenizer import build_tokenizer
    _G["tokenizer"] = build_tokenizer(args)
    return _G["tokenizer"]


def rebuild_tokenizer(args):
    _G["tokenizer"] = None
    return _build_tokenizer(args)


def _set_tensorboard_writer(args):
    """Writer lives on the last rank (reference global_vars.py:119-153)."""
    if args.rank != args.world_size - 1:
        return
    tb = None
    if getattr(args, "tensorboard_dir", None):
        try:
            from torch.utils.tensorboard import SummaryWriter
            print("> setting tensorboard ...", flush=True)
            tb = SummaryWriter(log_dir=args.tensorboard_dir, max_queue=args.tensorboard_queue_size)
        except Exception:
            print("WARNING: TensorBoard writing requested but is not available "
                  "(are you using PyTorch 1.1.0 or later?), no TensorBoard logs will be written.",
                  flush=True)
    if getattr(args, "wandb_logger", False):
        from .utils.wandb_logger import WandBConfig, WandbTBShim
        _G["tensorboard_writer"] = WandbTBShim(WandBConfig.from_args(args), tb)
    else:
        _G["tensorboard_writer"] = tb


def _set_adlr_autoresume(args):
    if not args.adlr_autoresume:
        return
    if args.rank == 0:
        print("enabling autoresume ...", flush=True)
    sys.path.append(os.environ.get("SUBMIT_SCRIPTS", "."))
    try:
        from userlib.auto_resume import AutoResume
    except ImportError:
        print("ADLR autoresume is not available, exiting ...")
        sys.exit()
    _G["adlr_autoresume"] = AutoResume


def _set_timers(args):
    _G["timers"] = Timers(args.timing_log_level, args.timing_log_option)


def reset_global_variables():
    for k in _G:
        _G[k] = None

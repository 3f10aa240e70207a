"""epfl_megatron_amd — MI355X-native 3D-parallel LLM training framework.

Feature parity target: the EPFL Megatron-LLM fork (andreaskoepf/epfl-megatron).
Compute path: PyTorch-ROCm + hand-written gfx950 HIP kernels (``csrc/``) +
RCCL over xGMI.  Public getters mirror ``megatron/__init__.py``.
"""
from .global_vars import (get_args, get_current_global_batch_size, get_num_microbatches,
                          get_signal_handler, update_num_microbatches, get_tokenizer,
                          get_tensorboard_writer, get_adlr_autoresume, get_timers)
from .utils.misc import print_rank_0, print_rank_last, is_last_rank

__version__ = "0.1.0"

"""Load Llama weights from a local Meta or Hugging Face directory as one
Meta-keyed state dict (reference ``weights2megatron/merge_llama.py``).

``merge_llama(size, version, root_dir) -> (state_dict, "meta" | "hf")``.
Meta model-parallel shards (``consolidated.NN.pth``) are concatenated along
each parameter's split axis; HF keys are renamed to Meta keys.  Only local
files are read (no downloads) and nothing is unpickled beyond tensors.
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), os.path.pardir)))

from epfl_megatron_amd.convert import hf_io  # noqa: E402
from epfl_megatron_amd.convert.llama import (META_SHARD_DIM as key_to_dim,  # noqa: E402,F401
                                             hf_to_meta, merge_meta_shards)


def merge_meta_llama(size, root_dir):
    return merge_meta_shards(hf_io.load_meta_shards(str(root_dir)))


def merge_hf_llama(size, version, cache_dir=None):
    if cache_dir is None:
        raise ValueError("a local Hugging Face model directory is required (no network)")
    return hf_to_meta(hf_io.load_hf_state_dict(str(cache_dir)))


def merge_llama(size, version, root_dir=None):
    if hf_io.is_meta_dir(str(root_dir) if root_dir else None):
        return merge_meta_llama(size, root_dir), "meta"
    print(f"Weights at {root_dir} do not look like a Meta checkpoint, assuming a Hugging Face "
          "directory instead")
    return merge_hf_llama(size, version, root_dir), "hf"

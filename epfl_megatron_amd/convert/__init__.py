"""Weight conversion between Meta / Hugging Face checkpoints and this framework.

Pure state-dict transforms (no model instantiation, no GPU) used by the CLI
scripts in ``weights2megatron/`` and ``tools/checkpoint_util.py``:

* :mod:`.qkv`      — fused-QKV packing and the RoPE row permutation;
* :mod:`.llama`    — Llama-1/2 (Meta ``consolidated.*.pth`` or HF) <-> Megatron;
* :mod:`.falcon`   — Falcon-7B/40B (HF) <-> Megatron;
* :mod:`.shard`    — tensor-parallel split/merge rules for re-sharding;
* :mod:`.megatron_ckpt` — read/write the on-disk Megatron checkpoint layout.
"""
from .qkv import permute_qkv, pack_qkv, unpack_qkv  # noqa: F401

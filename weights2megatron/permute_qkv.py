"""QKV row permutation (HF rotate-half <-> interleaved RoPE) and a migration
tool for old checkpoints (reference ``weights2megatron/permute_qkv.py``).

``python weights2megatron/permute_qkv.py --input-dir OLD --output-dir NEW``
rewrites every ``query_key_value.weight`` of every shard of the latest
iteration; ``--revert`` applies the inverse permutation.
"""
import argparse
import os
import re
import shutil
import sys
from pathlib import Path

import torch


sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), os.path.pardir)))

from epfl_megatron_amd import ckpt_pickle  # noqa: E402
from epfl_megatron_amd.checkpointing import safe_load  # noqa: E402
from epfl_megatron_amd.convert.qkv import permute_qkv  # noqa: E402,F401


def update_checkpoint(input_dir: Path, output_dir: Path, overwrite_ok=False, revert=False):
    input_dir, output_dir = Path(input_dir), Path(output_dir)
    if output_dir.exists():
        if not overwrite_ok:
            raise FileExistsError(f"Output directory {output_dir} already exists")
        shutil.rmtree(output_dir)
    output_dir.mkdir(parents=True)
    it = (input_dir / "latest_checkpointed_iteration.txt").read_text().strip()
    (output_dir / "latest_checkpointed_iteration.txt").write_text(it)
    sub = "release" if it == "release" else f"iter_{int(it):07d}"
    if not (input_dir / sub).is_dir() and (input_dir / it).is_dir():
        sub = it
    (output_dir / sub).mkdir()
    for shard in sorted((input_dir / sub).iterdir()):
        for f in sorted(shard.iterdir()):
            ck = safe_load(str(f))
            (output_dir / sub / shard.name).mkdir(exist_ok=True)
            if "model" in ck and "args" in ck:
                a = ck["args"]
                n_kv = getattr(a, "num_attention_heads_kv", None) or a.num_attention_heads
                lm = ck["model"]["language_model"]
                key = "transformer" if "transformer" in lm else "encoder"
                attn = "attention" if key == "transformer" else "self_attention"
                states = lm[key]
                for name in list(states):
                    if re.match(rf"^layers\.\d+\.{attn}\.query_key_value\.weight$", name):
                        states[name] = permute_qkv(states[name], a.hidden_size,
                                                   a.num_attention_heads, n_kv, revert=revert)
            torch.save(ck, output_dir / sub / shard.name / f.name,
                       pickle_module=ckpt_pickle.pickle_module)


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--input-dir", type=Path, required=True)
    p.add_argument("--output-dir", type=Path, required=True)
    p.add_argument("--overwrite-ok", action="store_true")
    p.add_argument("--revert", action="store_true")
    a = p.parse_args()
    update_checkpoint(a.input_dir, a.output_dir, a.overwrite_ok, a.revert)

"""Local checkpoint readers for conversion (no network, nothing unpickled).

* Hugging Face directories: ``*.safetensors`` (preferred) or
  ``pytorch_model*.bin`` read with ``torch.load(weights_only=True)``; the
  architecture comes from ``config.json``.
* Meta directories: ``consolidated.NN.pth`` shards (``weights_only=True``) and
  ``params.json``.
"""
import glob
import json
import os
import re

import torch


def read_json(path):
    with open(path) as f:
        return json.load(f)


def load_hf_state_dict(path):
    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if files:
        from safetensors.torch import load_file
        sd = {}
        for f in files:
            sd.update(load_file(f))
        return sd
    files = sorted(glob.glob(os.path.join(path, "pytorch_model*.bin")))
    if not files:
        raise FileNotFoundError(f"no *.safetensors or pytorch_model*.bin under {path}")
    sd = {}
    for f in files:
        sd.update(torch.load(f, map_location="cpu", weights_only=True))
    return sd


def hf_config(path):
    f = os.path.join(path, "config.json")
    return read_json(f) if os.path.isfile(f) else {}


def is_meta_dir(path):
    return path is not None and os.path.isfile(os.path.join(path, "consolidated.00.pth"))


def load_meta_shards(path):
    files = sorted(p for p in os.listdir(path) if re.match(r"^consolidated\.\d+\.pth$", p))
    return [torch.load(os.path.join(path, f), map_location="cpu", weights_only=True)
            for f in files]


def meta_params(path):
    f = os.path.join(path, "params.json")
    return read_json(f) if os.path.isfile(f) else {}

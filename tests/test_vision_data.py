"""Image folder dataset + AutoAugment policy (reference megatron/data/image_folder.py,
autoaugment.py); CPU, synthetic PNGs (the reference has no tests for these)."""
import random

import numpy as np
import pytest
import torch
from PIL import Image

from epfl_megatron_amd.data.vision import IMAGENET_POLICY, ImageFolder, ImageNetPolicy, to_tensor


def _make_tree(root):
    for c, n in (("cat", 4), ("dog", 2), ("eel", 3), ("fox", 5)):
        d = root / c
        d.mkdir()
        for i in range(n):
            Image.fromarray(np.full((8, 8, 3), 10 * i, np.uint8)).save(d / f"{i}.png")
        (d / "notes.txt").write_text("x")


def test_image_folder_fractions(tmp_path):
    _make_tree(tmp_path)
    ds = ImageFolder(str(tmp_path), transform=to_tensor)
    assert ds.classes == ["cat", "dog", "eel", "fox"] and len(ds) == 14
    img, t = ds[5]
    assert t == 1 and img.shape == (3, 8, 8) and img.dtype == torch.float32
    assert torch.allclose(img, torch.full_like(img, 10 / 255.0))
    half = ImageFolder(str(tmp_path), classes_fraction=0.5, data_per_class_fraction=0.5)
    assert half.classes == ["cat", "dog"]
    assert [(p.split("/")[-2:], t) for p, t in half.samples] == \
        [(["cat", "0.png"], 0), (["cat", "1.png"], 0), (["dog", "0.png"], 1)]


def test_autoaugment_policy():
    assert len(IMAGENET_POLICY) == 25
    random.seed(0)
    pol = ImageNetPolicy()
    rng = np.random.RandomState(0)
    img = Image.fromarray(rng.randint(0, 255, (32, 32, 3), dtype=np.uint8))
    changed = 0
    for _ in range(50):
        out = pol(img)
        assert out.size == img.size and out.mode == "RGB"
        changed += not np.array_equal(np.asarray(out), np.asarray(img))
    assert changed > 25
    # every op runs
    from epfl_megatron_amd.data.vision import SubPolicy
    for op in ("shearX", "shearY", "translateX", "translateY", "rotate", "color", "posterize",
               "solarize", "contrast", "sharpness", "brightness", "autocontrast", "equalize",
               "invert"):
        out = SubPolicy(1.0, op, 9, 0.0, "invert", 0)(img)
        assert out.size == img.size
    inv = SubPolicy(1.0, "invert", 0, 0.0, "invert", 0)(img)
    assert np.array_equal(np.asarray(inv), 255 - np.asarray(img))

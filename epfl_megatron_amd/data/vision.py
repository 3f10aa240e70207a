"""Image datasets and augmentation (reference ``megatron/data/image_folder.py``
and ``megatron/data/autoaugment.py``; not used by the language-model paths).

* ``ImageFolder`` — ``root/<class>/<image>`` layout, classes sorted
  alphabetically, with the reference's two sub-sampling knobs:
  ``classes_fraction`` keeps the first fraction of the sorted classes and
  ``data_per_class_fraction`` the first fraction of each class's sorted files
  (reference image_folder.py:64-110, 191-205).  torchvision is not in this
  image, so the dataset is a plain ``torch.utils.data.Dataset`` over PIL.
* ``ImageNetPolicy`` — the fixed 25-sub-policy AutoAugment ImageNet policy
  (Cubuk et al., 2019), each sub-policy two (operation, probability,
  magnitude bin) steps with 10 magnitude bins.
* ``to_tensor`` — PIL image -> float CHW tensor in [0, 1].
"""
import os
import random

import numpy as np
import torch
from PIL import Image, ImageEnhance, ImageOps

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def has_file_allowed_extension(filename, extensions):
    return filename.lower().endswith(tuple(extensions))


def is_image_file(filename):
    return has_file_allowed_extension(filename, IMG_EXTENSIONS)


def find_classes(directory, classes_fraction=1.0):
    names = sorted(e.name for e in os.scandir(directory) if e.is_dir())
    names = names[:int(len(names) * classes_fraction)]
    return names, {c: i for i, c in enumerate(names)}


def make_dataset(directory, class_to_idx, data_per_class_fraction=1.0, extensions=IMG_EXTENSIONS,
                 is_valid_file=None):
    if (extensions is None) == (is_valid_file is None):
        raise ValueError("Pass exactly one of extensions / is_valid_file")
    valid = is_valid_file or (lambda p: has_file_allowed_extension(p, extensions))
    out = []
    for cls in sorted(class_to_idx):
        files = []
        for root, _, names in sorted(os.walk(os.path.join(directory, cls), followlinks=True)):
            files += [(os.path.join(root, n), class_to_idx[cls]) for n in sorted(names)
                      if valid(os.path.join(root, n))]
        out += files[:int(len(files) * data_per_class_fraction)]
    return out


def pil_loader(path):
    with open(path, "rb") as f:
        return Image.open(f).convert("RGB")


class DatasetFolder(torch.utils.data.Dataset):
    def __init__(self, root, loader=pil_loader, extensions=IMG_EXTENSIONS, transform=None,
                 target_transform=None, is_valid_file=None, classes_fraction=1.0,
                 data_per_class_fraction=1.0):
        self.root, self.loader = root, loader
        self.transform, self.target_transform = transform, target_transform
        self.classes, self.class_to_idx = find_classes(root, classes_fraction)
        self.samples = make_dataset(root, self.class_to_idx, data_per_class_fraction,
                                    None if is_valid_file else extensions, is_valid_file)
        if not self.samples:
            raise RuntimeError(f"Found 0 files in subfolders of: {root}")
        self.targets = [t for _, t in self.samples]
        self.imgs = self.samples

    def __getitem__(self, index):
        path, target = self.samples[index]
        sample = self.loader(path)
        if self.transform is not None:
            sample = self.transform(sample)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return sample, target

    def __len__(self):
        return len(self.samples)


class ImageFolder(DatasetFolder):
    def __init__(self, root, transform=None, target_transform=None, loader=pil_loader,
                 is_valid_file=None, classes_fraction=1.0, data_per_class_fraction=1.0):
        super().__init__(root, loader, None if is_valid_file else IMG_EXTENSIONS, transform,
                         target_transform, is_valid_file, classes_fraction, data_per_class_fraction)


def to_tensor(img):
    a = np.asarray(img, dtype=np.float32) / 255.0
    if a.ndim == 2:
        a = a[:, :, None]
    return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))


# ---- AutoAugment ----------------------------------------------------------
_BINS = 10
_RANGES = {
    "shearX": np.linspace(0, 0.3, _BINS), "shearY": np.linspace(0, 0.3, _BINS),
    "translateX": np.linspace(0, 150 / 331, _BINS), "translateY": np.linspace(0, 150 / 331, _BINS),
    "rotate": np.linspace(0, 30, _BINS), "color": np.linspace(0.0, 0.9, _BINS),
    "posterize": np.round(np.linspace(8, 4, _BINS)).astype(int),
    "solarize": np.linspace(256, 0, _BINS), "contrast": np.linspace(0.0, 0.9, _BINS),
    "sharpness": np.linspace(0.0, 0.9, _BINS), "brightness": np.linspace(0.0, 0.9, _BINS),
    "autocontrast": [0] * _BINS, "equalize": [0] * _BINS, "invert": [0] * _BINS,
}


def _sign():
    return random.choice((-1, 1))


def _rotate_with_fill(img, deg):
    rot = img.convert("RGBA").rotate(deg)
    return Image.composite(rot, Image.new("RGBA", rot.size, (128,) * 4), rot).convert(img.mode)


def _ops(fill):
    aff = dict(fillcolor=fill)
    return {
        "shearX": lambda im, m: im.transform(im.size, Image.AFFINE, (1, m * _sign(), 0, 0, 1, 0),
                                             Image.BICUBIC, **aff),
        "shearY": lambda im, m: im.transform(im.size, Image.AFFINE, (1, 0, 0, m * _sign(), 1, 0),
                                             Image.BICUBIC, **aff),
        "translateX": lambda im, m: im.transform(
            im.size, Image.AFFINE, (1, 0, m * im.size[0] * _sign(), 0, 1, 0), **aff),
        "translateY": lambda im, m: im.transform(
            im.size, Image.AFFINE, (1, 0, 0, 0, 1, m * im.size[1] * _sign()), **aff),
        "rotate": lambda im, m: _rotate_with_fill(im, m * _sign()),
        "color": lambda im, m: ImageEnhance.Color(im).enhance(1 + m * _sign()),
        "posterize": lambda im, m: ImageOps.posterize(im, int(m)),
        "solarize": lambda im, m: ImageOps.solarize(im, m),
        "contrast": lambda im, m: ImageEnhance.Contrast(im).enhance(1 + m * _sign()),
        "sharpness": lambda im, m: ImageEnhance.Sharpness(im).enhance(1 + m * _sign()),
        "brightness": lambda im, m: ImageEnhance.Brightness(im).enhance(1 + m * _sign()),
        "autocontrast": lambda im, m: ImageOps.autocontrast(im),
        "equalize": lambda im, m: ImageOps.equalize(im),
        "invert": lambda im, m: ImageOps.invert(im),
    }


class SubPolicy:
    """Apply op1 with probability p1, then op2 with probability p2."""

    def __init__(self, p1, op1, bin1, p2, op2, bin2, fillcolor=(128, 128, 128)):
        ops = _ops(fillcolor)
        self.steps = [(p1, op1, ops[op1], _RANGES[op1][bin1]), (p2, op2, ops[op2], _RANGES[op2][bin2])]

    def __call__(self, img):
        for p, _, fn, mag in self.steps:
            if random.random() < p:
                img = fn(img, mag)
        return img

    def __repr__(self):
        return "SubPolicy(" + ", ".join(f"{n} p={p} m={m}" for p, n, _, m in self.steps) + ")"


IMAGENET_POLICY = [
    (0.4, "posterize", 8, 0.6, "rotate", 9), (0.6, "solarize", 5, 0.6, "autocontrast", 5),
    (0.8, "equalize", 8, 0.6, "equalize", 3), (0.6, "posterize", 7, 0.6, "posterize", 6),
    (0.4, "equalize", 7, 0.2, "solarize", 4), (0.4, "equalize", 4, 0.8, "rotate", 8),
    (0.6, "solarize", 3, 0.6, "equalize", 7), (0.8, "posterize", 5, 1.0, "equalize", 2),
    (0.2, "rotate", 3, 0.6, "solarize", 8), (0.6, "equalize", 8, 0.4, "posterize", 6),
    (0.8, "rotate", 8, 0.4, "color", 0), (0.4, "rotate", 9, 0.6, "equalize", 2),
    (0.0, "equalize", 7, 0.8, "equalize", 8), (0.6, "invert", 4, 1.0, "equalize", 8),
    (0.6, "color", 4, 1.0, "contrast", 8), (0.8, "rotate", 8, 1.0, "color", 2),
    (0.8, "color", 8, 0.8, "solarize", 7), (0.4, "sharpness", 7, 0.6, "invert", 8),
    (0.6, "shearX", 5, 1.0, "equalize", 9), (0.4, "color", 0, 0.6, "equalize", 3),
    (0.4, "equalize", 7, 0.2, "solarize", 4), (0.6, "solarize", 5, 0.6, "autocontrast", 5),
    (0.6, "invert", 4, 1.0, "equalize", 8), (0.6, "color", 4, 1.0, "contrast", 8),
    (0.8, "equalize", 8, 0.6, "equalize", 3),
]


class ImageNetPolicy:
    """Randomly pick one of the 25 ImageNet AutoAugment sub-policies per image."""

    def __init__(self, fillcolor=(128, 128, 128)):
        self.policies = [SubPolicy(*p, fillcolor=fillcolor) for p in IMAGENET_POLICY]

    def __call__(self, img):
        return self.policies[random.randint(0, len(self.policies) - 1)](img)

    def __repr__(self):
        return "AutoAugment ImageNet Policy"

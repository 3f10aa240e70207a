"""Indexed token corpora on disk (reference ``megatron/data/indexed_dataset.py``).

Two on-disk layouts are supported, both byte-compatible with the reference
(SURVEY Appendix C):

* ``mmap`` (``MMIDIDX``, :341-585) — the production format.  ``<prefix>.idx``
  holds ``magic(9) | <Q version=1 | <B dtype code | <Q n | <Q n_doc_idx |
  int32 sizes[n] | int64 byte pointers[n] | int64 doc_idx[n_doc_idx]``;
  ``<prefix>.bin`` is the flat token array.  The reader maps both files once
  and hands out zero-copy numpy views.
* ``lazy`` / ``cached`` (``TNTIDX``, :128-338) — the legacy fairseq layout
  (index of dim/data offsets, file reads per item).  Kept so that old corpora
  still load; new corpora should be ``mmap``.

Design notes (not a port): a single :class:`_MMapIndex` parses the header with
one ``np.frombuffer`` per section, item lookups are plain array indexing (no
``lru_cache`` tuples), and :meth:`MMapIndexedDataset.stitch` assembles whole
training samples that span documents in the native helper (``_helpers``)
straight out of the mapped ``.bin`` — the GPT dataset uses it so that sample
construction never goes through a per-document Python loop.
"""
import os
import shutil
import struct

import numpy as np
import torch

from ..utils.misc import print_rank_0

# dtype codes of the index header (reference :93-102) — part of the format.
DTYPES = {1: np.uint8, 2: np.int8, 3: np.int16, 4: np.int32, 5: np.int64,
          6: np.float32, 7: np.float64, 8: np.uint16}
_CODE_OF = {np.dtype(v): k for k, v in DTYPES.items()}

MMAP_MAGIC = b"MMIDIDX\x00\x00"
LEGACY_MAGIC = b"TNTIDX\x00\x00"


def code(dtype):
    try:
        return _CODE_OF[np.dtype(dtype)]
    except KeyError:
        raise ValueError(f"unsupported token dtype {dtype}") from None


def best_fitting_dtype(vocab_size=None):
    """uint16 when every id fits (vocab < 65500), else int32 (reference :24-28)."""
    return np.uint16 if vocab_size is not None and vocab_size < 65500 else np.int32


def index_file_path(prefix):
    return prefix + ".idx"


def data_file_path(prefix):
    return prefix + ".bin"


def get_available_dataset_impl():
    return ["lazy", "cached", "mmap"]


def _exists(prefix):
    return os.path.exists(index_file_path(prefix)) and os.path.exists(data_file_path(prefix))


def infer_dataset_impl(path):
    if not _exists(path):
        print(f"Dataset does not exist: {path} (expected {path}.idx and {path}.bin)")
        return None
    with open(index_file_path(path), "rb") as f:
        magic = f.read(9)
    if magic == MMAP_MAGIC:
        return "mmap"
    if magic[:8] == LEGACY_MAGIC:
        return "cached"
    return None


def make_builder(out_file, impl, vocab_size=None):
    if impl == "mmap":
        return MMapIndexedDatasetBuilder(out_file, dtype=best_fitting_dtype(vocab_size))
    return IndexedDatasetBuilder(out_file)


def make_dataset(path, impl, skip_warmup=False):
    if not _exists(path):
        print(f"Dataset does not exist: {path} (expected {path}.idx and {path}.bin)")
        return None
    if impl == "infer":
        impl = infer_dataset_impl(path)
    if impl == "lazy":
        return IndexedDataset(path)
    if impl == "cached":
        return IndexedCachedDataset(path)
    if impl == "mmap":
        return MMapIndexedDataset(path, skip_warmup)
    print(f"Unknown dataset implementation: {impl}")
    return None


def dataset_exists(path, impl):
    return _exists(path)


def _warmup(path, chunk=100 << 20):
    with open(path, "rb") as f:
        while f.read(chunk):
            pass


def create_doc_idx(sizes):
    """Legacy helper: an empty item separates documents."""
    return [0] + [i + 1 for i, s in enumerate(sizes) if s == 0]


# --------------------------------------------------------------------------- mmap
class _MMapIndex:
    """Parsed ``.idx`` of the mmap layout: sizes / pointers / doc_idx views."""

    def __init__(self, path, skip_warmup=False):
        with open(path, "rb") as f:
            head = f.read(9 + 8 + 1 + 8 + 8)
        if head[:9] != MMAP_MAGIC:
            raise ValueError(f"{path}: not an MMIDIDX index (check --data_impl)")
        version, = struct.unpack_from("<Q", head, 9)
        if version != 1:
            raise ValueError(f"{path}: unsupported index version {version}")
        self.dtype = DTYPES[head[17]]
        n, n_doc = struct.unpack_from("<QQ", head, 18)
        if not skip_warmup:
            print_rank_0("    warming up index mmap file...")
            _warmup(path)
        self._mm = np.memmap(path, mode="r", order="C")
        off = 34
        self.sizes = np.frombuffer(self._mm, dtype=np.int32, count=n, offset=off)
        off += 4 * n
        self.pointers = np.frombuffer(self._mm, dtype=np.int64, count=n, offset=off)
        off += 8 * n
        self.doc_idx = np.frombuffer(self._mm, dtype=np.int64, count=n_doc, offset=off)

    def __len__(self):
        return self.sizes.shape[0]

    def __getitem__(self, i):
        return int(self.pointers[i]), int(self.sizes[i])

    @staticmethod
    def write(path, dtype, sizes, doc_idx):
        sizes = np.asarray(sizes, dtype=np.int32)
        itemsize = np.dtype(dtype).itemsize
        pointers = np.zeros(sizes.shape[0], dtype=np.int64)
        if sizes.shape[0] > 1:
            np.cumsum(sizes[:-1].astype(np.int64) * itemsize, out=pointers[1:])
        doc_idx = np.asarray(doc_idx, dtype=np.int64)
        with open(path, "wb") as f:
            f.write(MMAP_MAGIC)
            f.write(struct.pack("<Q", 1))
            f.write(struct.pack("<B", code(dtype)))
            f.write(struct.pack("<QQ", sizes.shape[0], doc_idx.shape[0]))
            f.write(sizes.tobytes(order="C"))
            f.write(pointers.tobytes(order="C"))
            f.write(doc_idx.tobytes(order="C"))


class MMapIndexedDataset(torch.utils.data.Dataset):
    """Zero-copy reader of ``<prefix>.idx/.bin`` (reference :341-544)."""

    Index = _MMapIndex

    def __init__(self, path, skip_warmup=False):
        super().__init__()
        self._open(path, skip_warmup)

    def _open(self, path, skip_warmup=True):
        self._path = path
        self._index = _MMapIndex(index_file_path(path), skip_warmup)
        if not skip_warmup:
            print_rank_0("    warming up data mmap file...")
            _warmup(data_file_path(path))
        self._bin = np.memmap(data_file_path(path), mode="r", order="C")
        self._tokens = None

    # DataLoader workers re-open the maps instead of pickling them.
    def __getstate__(self):
        return self._path

    def __setstate__(self, path):
        self._open(path, True)

    def __len__(self):
        return len(self._index)

    @property
    def dtype(self):
        return self._index.dtype

    @property
    def sizes(self):
        return self._index.sizes

    @property
    def doc_idx(self):
        return self._index.doc_idx

    def get_doc_idx(self):
        return self._index.doc_idx

    def set_doc_idx(self, doc_idx):
        self._index.doc_idx = doc_idx

    @property
    def supports_prefetch(self):
        return False

    @staticmethod
    def exists(path):
        return _exists(path)

    @property
    def tokens(self):
        """The whole ``.bin`` as one flat token array (a view of the map)."""
        if self._tokens is None:
            self._tokens = np.frombuffer(self._bin, dtype=self.dtype)
        return self._tokens

    def __getitem__(self, idx):
        if isinstance(idx, (int, np.integer)):
            return self.get(int(idx))
        if isinstance(idx, slice):
            start, stop, step = idx.indices(len(self))
            if step != 1:
                raise ValueError("slices into an indexed dataset must be contiguous")
            sizes = self._index.sizes[start:stop]
            base = int(self._index.pointers[start]) // np.dtype(self.dtype).itemsize
            flat = self.tokens[base:base + int(sizes.sum())]
            return np.split(flat, np.cumsum(sizes)[:-1])
        raise TypeError(f"unexpected index type {type(idx)}")

    def get(self, idx, offset=0, length=None):
        """Tokens ``[offset, offset+length)`` of item ``idx`` (a view)."""
        ptr, size = self._index[idx]
        if length is None:
            length = size - offset
        start = ptr // np.dtype(self.dtype).itemsize + offset
        return self.tokens[start:start + length]

    def stitch(self, doc_idx, sample_idx, samples, seq_length):
        """Native assembly of GPT samples ``samples`` -> int64 ``[len, seq_length+1]``.

        ``sample_idx[i] = (position in doc_idx, token offset)`` as built by
        ``helpers.build_sample_idx``; sample ``i`` runs from ``sample_idx[i]``
        to ``sample_idx[i+1]`` inclusive (reference ``gpt_dataset.py:243-269``).
        """
        from . import helpers
        return helpers.stitch_samples(self.tokens, self._index.pointers, self._index.sizes,
                                      doc_idx, sample_idx, samples, seq_length)


class MMapIndexedDatasetBuilder:
    """Streaming writer for the mmap layout (reference :547-585)."""

    def __init__(self, out_file, dtype=np.int64):
        self._file = open(out_file, "wb")
        self._dtype = np.dtype(dtype).type
        self._sizes = []
        self._doc_idx = [0]

    def add_item(self, tensor):
        arr = np.asarray(tensor.numpy() if torch.is_tensor(tensor) else tensor, dtype=self._dtype)
        self._file.write(arr.tobytes(order="C"))
        self._sizes.append(arr.size)

    def add_doc(self, tokens, sizes):
        arr = np.asarray(tokens, dtype=self._dtype)
        self._file.write(arr.tobytes(order="C"))
        self._sizes.extend(int(s) for s in sizes)
        self._doc_idx.append(len(self._sizes))

    def end_document(self):
        self._doc_idx.append(len(self._sizes))

    def merge_file_(self, another_prefix):
        idx = _MMapIndex(index_file_path(another_prefix), skip_warmup=True)
        if np.dtype(idx.dtype) != np.dtype(self._dtype):
            raise ValueError(f"dtype mismatch merging {another_prefix}: {idx.dtype} vs {self._dtype}")
        base = len(self._sizes)
        self._sizes.extend(idx.sizes.tolist())
        self._doc_idx.extend((base + idx.doc_idx[1:]).tolist())
        with open(data_file_path(another_prefix), "rb") as f:
            shutil.copyfileobj(f, self._file)

    def finalize(self, index_file):
        self._file.close()
        _MMapIndex.write(index_file, self._dtype, self._sizes, self._doc_idx)


# ------------------------------------------------------------------------- legacy
_LEGACY_ELEMENT_SIZE = {np.uint8: 1, np.int8: 1, np.int16: 2, np.int32: 4, np.int64: 8,
                        np.float32: 4, np.float64: 8, np.uint16: 2}


class IndexedDataset(torch.utils.data.Dataset):
    """Legacy ``TNTIDX`` reader, reads items from the file on demand (reference :128-209)."""

    _HDR_MAGIC = LEGACY_MAGIC

    def __init__(self, path):
        super().__init__()
        self.path = path
        self.data_file = None
        with open(index_file_path(path), "rb") as f:
            if f.read(8) != LEGACY_MAGIC:
                raise ValueError(f"{path}: not a TNTIDX index (check --data_impl)")
            version, = struct.unpack("<Q", f.read(8))
            assert version == 1
            dcode, self.element_size = struct.unpack("<QQ", f.read(16))
            self.dtype = DTYPES[dcode]
            self._len, n_sizes = struct.unpack("<QQ", f.read(16))
            n_doc, = struct.unpack("<Q", f.read(8))
            rest = np.frombuffer(f.read(), dtype=np.int64)
        n = self._len + 1
        self.dim_offsets = rest[:n]
        self.data_offsets = rest[n:2 * n]
        self.sizes = rest[2 * n:2 * n + n_sizes]
        self.doc_idx = rest[2 * n + n_sizes:2 * n + n_sizes + n_doc]

    def _read(self, start, count):
        if self.data_file is None:
            self.data_file = open(data_file_path(self.path), "rb", buffering=0)
        a = np.empty(count, dtype=self.dtype)
        self.data_file.seek(int(start) * self.element_size)
        self.data_file.readinto(a)
        return a

    def __del__(self):
        if getattr(self, "data_file", None):
            self.data_file.close()

    def _item(self, i):
        if i < 0 or i >= self._len:
            raise IndexError("index out of range")
        shape = self.sizes[self.dim_offsets[i]:self.dim_offsets[i + 1]]
        return self._read(self.data_offsets[i], int(np.prod(shape))).reshape(shape)

    def __getitem__(self, idx):
        if isinstance(idx, (int, np.integer)):
            return self._item(int(idx))
        start, stop, step = idx.indices(len(self))
        if step != 1:
            raise ValueError("slices into an indexed dataset must be contiguous")
        return [self._item(i) for i in range(start, stop)]

    def get(self, idx, offset=0, length=None):
        a = self._item(idx)
        return a[offset:] if length is None else a[offset:offset + length]

    def __len__(self):
        return self._len

    def num_tokens(self, index):
        return self.sizes[index]

    def size(self, index):
        return self.sizes[index]

    @staticmethod
    def exists(path):
        return _exists(path)

    @property
    def supports_prefetch(self):
        return False


class IndexedCachedDataset(IndexedDataset):
    """Legacy reader that prefetches the requested items into RAM (reference :212-262)."""

    def __init__(self, path):
        super().__init__(path)
        self.cache = {}

    @property
    def supports_prefetch(self):
        return True

    def prefetch(self, indices):
        for i in sorted(set(int(i) for i in indices)):
            if i not in self.cache:
                self.cache[i] = IndexedDataset._item(self, i)
        if self.data_file:
            self.data_file.close()
            self.data_file = None

    def _item(self, i):
        if i in self.cache:
            return self.cache[i].copy()
        return IndexedDataset._item(self, i)


class IndexedDatasetBuilder:
    """Legacy ``TNTIDX`` writer (reference :265-338)."""

    def __init__(self, out_file, dtype=np.int32):
        self.out_file = open(out_file, "wb")
        self.dtype = np.dtype(dtype).type
        self.element_size = _LEGACY_ELEMENT_SIZE[self.dtype]
        self.data_offsets = [0]
        self.dim_offsets = [0]
        self.sizes = []
        self.doc_idx = [0]

    def add_item(self, tensor):
        arr = np.asarray(tensor.numpy() if torch.is_tensor(tensor) else tensor, dtype=self.dtype)
        self.out_file.write(arr.tobytes(order="C"))
        self.data_offsets.append(self.data_offsets[-1] + arr.size)
        self.sizes.extend(arr.shape)
        self.dim_offsets.append(self.dim_offsets[-1] + arr.ndim)

    def end_document(self):
        self.doc_idx.append(len(self.sizes))

    def merge_file_(self, another_prefix):
        other = IndexedDataset(another_prefix)
        assert np.dtype(other.dtype) == np.dtype(self.dtype)
        doc_base = len(self.sizes)
        base = self.data_offsets[-1]
        self.data_offsets.extend((base + other.data_offsets[1:]).tolist())
        self.sizes.extend(other.sizes.tolist())
        base = self.dim_offsets[-1]
        self.dim_offsets.extend((base + other.dim_offsets[1:]).tolist())
        self.doc_idx.extend((doc_base + other.doc_idx[1:]).tolist())
        with open(data_file_path(another_prefix), "rb") as f:
            shutil.copyfileobj(f, self.out_file)

    def finalize(self, index_file):
        self.out_file.close()
        with open(index_file, "wb") as f:
            f.write(LEGACY_MAGIC)
            f.write(struct.pack("<Q", 1))
            f.write(struct.pack("<QQ", code(self.dtype), self.element_size))
            f.write(struct.pack("<QQ", len(self.data_offsets) - 1, len(self.sizes)))
            f.write(struct.pack("<Q", len(self.doc_idx)))
            for arr in (self.dim_offsets, self.data_offsets, self.sizes, self.doc_idx):
                f.write(np.asarray(arr, dtype=np.int64).tobytes())

"""Evidence-embedding store and maximum-inner-product search
(reference ``megatron/data/realm_index.py``: ``OpenRetreivalDataStore`` :17,
``FaissMIPSIndex`` :118).

MI355X design: there is no FAISS here.  A flat inner-product index is one
GEMM, so the whole evidence matrix is kept resident in HBM (21M DPR passages
x 768 dims in bf16 is ~32 GB, comfortably inside 288 GB) and queries are
scored with ``torch.mm`` on the matrix cores in row blocks, merging a running
top-k per block.  On CPU the same code runs in fp32.

Storage never uses pickle: each shard / the merged index is an ``.npz`` with
``ids`` (int64) and ``embeds`` (fp16), loaded with ``allow_pickle=False``.
"""
import os
import shutil

import numpy as np
import torch

from .. import global_vars
from ..parallel import state


def detach(tensor):
    return tensor.detach().cpu().numpy()


def _is_main():
    return not state.model_parallel_is_initialized() or state.get_data_parallel_rank() == 0


def _save_npz(path, embed_data):
    ids = np.fromiter(embed_data.keys(), dtype=np.int64, count=len(embed_data))
    emb = np.stack(list(embed_data.values())).astype(np.float16) if embed_data else \
        np.zeros((0, 0), np.float16)
    tmp = path + ".tmp.npz"
    np.savez(tmp, ids=ids, embeds=emb)
    os.replace(tmp, path)


def _load_npz(path):
    with np.load(path, allow_pickle=False) as z:
        return dict(zip(z["ids"].tolist(), z["embeds"]))


class OpenRetrievalDataStore:
    """id -> fp16 embedding, written per DP rank then merged by rank 0."""

    def __init__(self, embedding_path=None, load_from_path=True, rank=None):
        if embedding_path is None:
            args = global_vars.get_args()
            embedding_path, rank = args.embedding_path, args.rank
        self.embedding_path = embedding_path
        self.rank = rank
        self.embed_data = {}
        if load_from_path:
            self.load_from_file()
        self.temp_dir_name = os.path.splitext(self.embedding_path)[0] + "_tmp"

    def state(self):
        return {"embed_data": self.embed_data}

    def clear(self):
        self.embed_data = {}

    def load_from_file(self):
        if _is_main():
            print("\n> Loading evidence embeddings", flush=True)
        self.embed_data = _load_npz(self.embedding_path)
        if _is_main():
            print(f">> Loaded {len(self.embed_data)} embeddings\n", flush=True)

    def add_block_data(self, row_id, block_embeds, allow_overwrite=False):
        for idx, emb in zip(np.asarray(row_id).tolist(), block_embeds):
            if not allow_overwrite and idx in self.embed_data:
                raise ValueError("Unexpectedly tried to overwrite block data")
            self.embed_data[idx] = np.float16(emb)

    def save_shard(self):
        os.makedirs(self.temp_dir_name, exist_ok=True)
        _save_npz(os.path.join(self.temp_dir_name, f"{self.rank}.npz"), self.embed_data)

    def merge_shards_and_save(self):
        names = sorted(os.listdir(self.temp_dir_name))
        seen_own = False
        for fname in names:
            shard_rank = int(fname.split(".")[0])
            if shard_rank == self.rank:
                seen_own = True
                continue
            shard = _load_npz(os.path.join(self.temp_dir_name, fname))
            before = len(self.embed_data)
            self.embed_data.update(shard)
            assert len(self.embed_data) == before + len(shard), "duplicate ids across shards"
        assert seen_own
        _save_npz(self.embedding_path, self.embed_data)
        shutil.rmtree(self.temp_dir_name, ignore_errors=True)
        print(f"Finished merging {len(names)} shards for a total of {len(self.embed_data)} "
              "embeds", flush=True)


# reference spelling
OpenRetreivalDataStore = OpenRetrievalDataStore


class MIPSIndex:
    """Exact flat inner-product index, resident on the device.

    ``search_mips_index(q, k, reconstruct=False)`` -> ``(scores [n,k] fp32,
    ids [n,k] int64)`` as numpy (FAISS ``IndexIDMap(IndexFlatIP)`` contract);
    with ``reconstruct=True`` also the ``[n,k,d]`` embeddings of the hits.
    """

    def __init__(self, embed_size, embed_data=None, use_gpu=None, block_rows=1 << 20):
        self.embed_size = embed_size
        self.embed_data = embed_data
        if use_gpu is None:
            use_gpu = torch.cuda.is_available()
        self.device = torch.device("cuda", torch.cuda.current_device()) if use_gpu and \
            torch.cuda.is_available() else torch.device("cpu")
        # bf16 operands on MFMA with fp32 accumulation; fp32 on the CPU path
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.block_rows = block_rows
        self.reset_storage()
        if embed_data is not None:
            self.add_embed_data(embed_data)

    def reset_storage(self):
        self.ids = torch.zeros(0, dtype=torch.int64, device=self.device)
        self.embeds = torch.zeros(0, self.embed_size, dtype=self.dtype, device=self.device)

    def reset_index(self):
        path = self.embed_data.embedding_path if self.embed_data is not None else None
        self.reset_storage()
        if path is not None:
            self.embed_data = OpenRetrievalDataStore(path)
            self.add_embed_data(self.embed_data)

    def update_index(self):
        self.reset_storage()
        if self.embed_data is not None:
            self.embed_data.load_from_file()
            self.add_embed_data(self.embed_data)

    def add_embed_data(self, all_embed_data):
        data = all_embed_data.embed_data if hasattr(all_embed_data, "embed_data") \
            else all_embed_data
        if not data:
            return
        ids = torch.as_tensor(np.fromiter(data.keys(), dtype=np.int64, count=len(data)))
        emb = torch.from_numpy(np.stack(list(data.values())).astype(np.float32))
        assert emb.shape[1] == self.embed_size, (emb.shape, self.embed_size)
        if hasattr(all_embed_data, "clear"):
            all_embed_data.clear()
        self.ids = torch.cat([self.ids, ids.to(self.device)])
        self.embeds = torch.cat([self.embeds, emb.to(self.device, self.dtype)])
        if _is_main():
            print(">>> Finished adding block data to index", flush=True)

    @torch.no_grad()
    def _topk(self, q, k):
        q = q.to(self.device, self.dtype)
        n = self.embeds.shape[0]
        k = min(k, n)
        best_s = torch.full((q.shape[0], 0), float("-inf"), device=self.device)
        best_i = torch.zeros((q.shape[0], 0), dtype=torch.int64, device=self.device)
        for start in range(0, n, self.block_rows):
            blk = self.embeds[start:start + self.block_rows]
            s = torch.mm(q, blk.t()).float()
            kk = min(k, s.shape[1])
            s, i = torch.topk(s, kk, dim=1)
            best_s = torch.cat([best_s, s], 1)
            best_i = torch.cat([best_i, i + start], 1)
            if best_s.shape[1] > k:
                best_s, sel = torch.topk(best_s, k, dim=1)
                best_i = torch.gather(best_i, 1, sel)
        return best_s, best_i

    def search_mips_index(self, query_embeds, top_k, reconstruct=True):
        q = torch.as_tensor(query_embeds).float()
        scores, rows = self._topk(q, top_k)
        ids = self.ids[rows]
        if reconstruct:
            return self.embeds[rows].float().cpu().numpy()
        return scores.cpu().numpy(), ids.cpu().numpy()


# reference name (the FAISS wrapper); same contract, device-resident GEMM search
FaissMIPSIndex = MIPSIndex

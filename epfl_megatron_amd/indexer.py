"""Evidence-embedding index builder (reference ``megatron/indexer.py:17-123``).

One pass of the context tower over the evidence passages, each DP rank
embedding its slice; every rank writes an ``.npz`` shard and DP-rank 0 merges
them into ``--embedding_path`` (see ``data/realm_index.py``).
"""
import torch
import torch.distributed as dist

from . import checkpointing, global_vars, training
from .data.orqa_wiki_dataset import (get_one_epoch_dataloader, get_open_retrieval_batch,
                                     get_open_retrieval_wiki_dataset)
from .data.realm_index import OpenRetrievalDataStore, detach
from .models import ModelType
from .models.biencoder_model import get_model_provider
from .parallel import state


class IndexBuilder:
    def __init__(self, args=None):
        args = args or global_vars.get_args()
        self.shared = args.biencoder_shared_query_context_model
        assert not (args.load and args.ict_load), "give either --load or --ict_load"
        self.log_interval = args.indexer_log_interval
        self.batch_size = args.indexer_batch_size
        self.is_main_builder = state.get_data_parallel_rank() == 0
        self.num_total_builders = state.get_data_parallel_world_size()
        self.iteration = self.total_processed = 0
        self.load_attributes(args)

    def load_attributes(self, args):
        only_context = not self.shared
        provider = get_model_provider(only_context_model=only_context,
                                      biencoder_shared_query_context_model=self.shared)
        model = training.get_model(provider, ModelType.encoder_or_decoder, wrap_with_ddp=False,
                                   args=args)
        load_path = args.load or args.ict_load
        self.model = checkpointing.load_biencoder_checkpoint(
            model, only_context_model=only_context, custom_load_path=load_path)
        assert len(self.model) == 1
        self.model[0].eval()
        self.dataset = get_open_retrieval_wiki_dataset()
        self.dataloader = iter(get_one_epoch_dataloader(self.dataset, self.batch_size))
        self.evidence_embedder_obj = OpenRetrievalDataStore(load_from_path=False)

    def track_and_report_progress(self, batch_size):
        self.iteration += 1
        self.total_processed += batch_size * self.num_total_builders
        if self.is_main_builder and self.iteration % self.log_interval == 0:
            print(f"Batch {self.iteration:10d} | Total {self.total_processed:10d}", flush=True)

    @torch.no_grad()
    def build_and_save_index(self):
        m = self.model[0]
        while not hasattr(m, "embed_text"):
            m = m.module
        while True:
            try:
                row_id, ctx, ctx_mask, ctx_types, _ = get_open_retrieval_batch(self.dataloader)
            except (StopIteration, IndexError):
                break
            assert ctx_mask.dtype == torch.bool
            dev = next(m.parameters()).device
            emb = m.embed_text(m.context_model, ctx.to(dev), ctx_mask.to(dev), ctx_types.to(dev))
            self.evidence_embedder_obj.add_block_data(detach(row_id), detach(emb.float()))
            self.track_and_report_progress(len(row_id))
        self.evidence_embedder_obj.save_shard()
        if dist.is_initialized():
            dist.barrier()
        del self.model
        if self.is_main_builder:
            self.evidence_embedder_obj.merge_shards_and_save()
            assert len(self.evidence_embedder_obj.embed_data) == len(self.dataset)
        self.evidence_embedder_obj.clear()
        if dist.is_initialized():
            dist.barrier()

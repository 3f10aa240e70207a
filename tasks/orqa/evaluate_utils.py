"""Zero-shot retrieval evaluation (reference ``tasks/orqa/evaluate_utils.py``).

Queries are embedded by the query tower, all-gathered over the world, and
searched against the device-resident evidence index (``MIPSIndex``).  Unlike
the reference (FAISS on local rank 0 of each node, then broadcast), every rank
holds the index in HBM and searches only its own queries — 288 GB per GPU
leaves room for the full DPR Wikipedia index next to the model — so no
per-node groups or broadcasts are needed.  Answer matching then runs on the
CPU (``qa_utils.calculate_matches``).
"""
import torch

from epfl_megatron_amd import checkpointing, get_args, print_rank_0
from epfl_megatron_amd.data.orqa_wiki_dataset import get_open_retrieval_wiki_dataset
from epfl_megatron_amd.data.realm_index import MIPSIndex, OpenRetrievalDataStore
from epfl_megatron_amd.models import ModelType
from epfl_megatron_amd.models.biencoder_model import get_model_provider
from epfl_megatron_amd.training import get_model

from .unsupervised.nq import get_nq_dataset, get_one_epoch_nq_dataloader, process_nq_batch
from .unsupervised.qa_utils import calculate_matches


class ORQAEvaluator:
    def __init__(self):
        args = get_args()
        self.embedding_size = args.biencoder_projection_dim or args.hidden_size
        self.evidence_dataset = get_open_retrieval_wiki_dataset()
        only_query = not args.biencoder_shared_query_context_model
        provider = get_model_provider(
            only_query_model=only_query,
            biencoder_shared_query_context_model=args.biencoder_shared_query_context_model,
            model_type=ModelType.encoder_or_decoder)
        model = get_model(provider, ModelType.encoder_or_decoder, wrap_with_ddp=False, args=args)
        self.model = checkpointing.load_biencoder_checkpoint(model, only_query_model=only_query)
        assert len(self.model) == 1
        self.model[0].eval()
        self.mips_index = MIPSIndex(self.embedding_size,
                                    OpenRetrievalDataStore(load_from_path=True),
                                    use_gpu=torch.cuda.is_available())

    @torch.no_grad()
    def generate_query_vectors(self, qa_data, split):
        self.eval_dataset = get_nq_dataset(qa_data, split)
        m = self.model[0]
        while not hasattr(m, "embed_text"):
            m = m.module
        vecs, refs = [], []
        for batch in get_one_epoch_nq_dataloader(self.eval_dataset):
            tokens, mask, types, _, reference = process_nq_batch(batch)
            vecs.append(m.embed_text(m.query_model, tokens, mask, types).float())
            refs.extend(reference)
        q = torch.cat(vecs)
        assert q.size(0) == len(self.eval_dataset)
        print_rank_0(f"Total encoded queries tensor {tuple(q.size())}")
        return q, refs

    def evaluate(self, qa_data, split):
        args = get_args()
        q, refs = self.generate_query_vectors(qa_data, split)
        scores, ids = self.mips_index.search_mips_index(q, args.faiss_topk_retrievals,
                                                        reconstruct=False)
        top = [(i.tolist(), s.tolist()) for i, s in zip(ids, scores)]
        stats = calculate_matches(self.evidence_dataset.id2text, refs, top,
                                  workers_num=args.num_workers, match_type=args.faiss_match)
        hits = stats.top_k_hits
        print_rank_0(f"{split} SET RESULTS")
        print_rank_0(f"topk-{args.faiss_topk_retrievals} documents hits {hits}")
        acc = [v / len(top) for v in hits]
        print_rank_0(f"top-k documents hits accuracy {acc}")
        for k in args.retriever_report_topk_accuracies:
            print_rank_0(f"top-{k}: {acc[k - 1] * 100:.2f}")
        return acc

"""ICT-ZEROSHOT-NQ / RETRIEVER-EVAL (reference ``tasks/orqa/evaluate_orqa.py``):
embed the evidence with the context tower (``IndexBuilder``), then score NQ
dev/test retrieval with the query tower."""
from epfl_megatron_amd import get_args, print_rank_0
from epfl_megatron_amd.indexer import IndexBuilder

from .evaluate_utils import ORQAEvaluator


def main():
    args = get_args()
    print_rank_0("Starting index builder!")
    IndexBuilder(args).build_and_save_index()
    print_rank_0("Build and save indices: done!")
    print_rank_0("Starting evaluations!")
    evaluator = ORQAEvaluator()
    out = {}
    if args.qa_data_dev is not None:
        out["DEV"] = evaluator.evaluate(args.qa_data_dev, "DEV")
    if args.qa_data_test is not None:
        out["TEST"] = evaluator.evaluate(args.qa_data_test, "TEST")
    return out

"""Downstream task entry point (reference tasks/main.py).

    python tasks/main.py --task {LAMBADA,WIKITEXT103} --valid_data FILE --load CKPT \
        --model_name llama2 ... [--overlapping_eval 32] [--strict_lambada]

The GPT-family zero-shot tasks are implemented; the BERT-based finetuning
tasks of the reference (RACE, MNLI, QQP, ICT / retriever) are legacy and
are rejected with a clear error.
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), os.path.pardir)))

from epfl_megatron_amd import get_args  # noqa: E402
from epfl_megatron_amd.initialize import initialize_megatron  # noqa: E402


def get_tasks_args(parser):
    import finetune
    parser = finetune.extra_args(parser)
    g = parser.add_argument_group(title="tasks")
    g.add_argument("--task", type=str, required=True)
    g.add_argument("--epochs", type=int, default=None)
    g.add_argument("--pretrained_checkpoint", type=str, default=None)
    g.add_argument("--keep_last", action="store_true")
    g.add_argument("--train_data", nargs="+", default=None)
    g.add_argument("--valid_data", nargs="*", default=None)
    g.add_argument("--overlapping_eval", type=int, default=32)
    g.add_argument("--strict_lambada", action="store_true")
    g.add_argument("--qa_data_dev", type=str, default=None)
    g.add_argument("--qa_data_test", type=str, default=None)
    g.add_argument("--faiss_use_gpu", action="store_true")
    g.add_argument("--faiss_match", type=str, default="string", choices=["regex", "string"])
    g.add_argument("--faiss_topk_retrievals", type=int, default=100)
    g.add_argument("--eval_micro_batch_size", type=int, default=None)
    g.add_argument("--train_with_neg", action="store_true")
    g.add_argument("--train_hard_neg", type=int, default=0)
    g.add_argument("--val_av_rank_hard_neg", type=int, default=30)
    g.add_argument("--val_av_rank_other_neg", type=int, default=30)
    return parser


def main(argv=None):
    initialize_megatron(get_tasks_args, args_list=argv)
    args = get_args()
    if args.num_layers_per_virtual_pipeline_stage is not None:
        raise SystemExit("Interleaved pipeline schedule is not supported for downstream tasks.")
    if args.task in ("LAMBADA", "WIKITEXT103"):
        from tasks.zeroshot_gpt.evaluate import main as zeroshot
        return zeroshot()
    if args.task in ("RACE", "MNLI", "QQP", "ICT-ZEROSHOT-NQ", "RETRIEVER-EVAL",
                     "RET-FINETUNE-NQ"):
        raise NotImplementedError(f"{args.task} is a BERT-family task (legacy in the "
                                  "reference); only GPT-family zero-shot tasks are provided")
    raise NotImplementedError(f"Task {args.task} is not implemented.")


if __name__ == "__main__":
    main()

"""Downstream task entry point (reference tasks/main.py).

    python tasks/main.py --task {LAMBADA,WIKITEXT103} --valid_data FILE --load CKPT \
        --model_name llama2 ... [--overlapping_eval 32] [--strict_lambada]

Dispatch (reference tasks/main.py:82-94): RACE -> tasks.race, MNLI/QQP ->
tasks.glue, LAMBADA/WIKITEXT103 -> tasks.zeroshot_gpt, ICT-ZEROSHOT-NQ /
RETRIEVER-EVAL -> tasks.orqa.evaluate_orqa, RET-FINETUNE-NQ ->
tasks.orqa.supervised.finetune.
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
    if args.task == "RACE":
        from tasks.race.finetune import main as race
        return race()
    if args.task in ("MNLI", "QQP"):
        from tasks.glue.finetune import main as glue
        return glue()
    if args.task in ("ICT-ZEROSHOT-NQ", "RETRIEVER-EVAL"):
        from tasks.orqa.evaluate_orqa import main as orqa_eval
        return orqa_eval()
    if args.task == "RET-FINETUNE-NQ":
        from tasks.orqa.supervised.finetune import main as ret_finetune
        return ret_finetune()
    raise NotImplementedError(f"Task {args.task} is not implemented.")


if __name__ == "__main__":
    main()

"""Multi-stage dialogue prompting entry point (reference ``tasks/msdp/main.py``).

    python tasks/msdp/main.py --task MSDP-PROMPT --prompt_type knowledge \
        --prompt_file P.jsonl --sample_input_file test.tsv --sample_output_file out.txt \
        --load CKPT --model_name llama2 ...
    python tasks/msdp/main.py --task MSDP-EVAL-F1 --guess_file out.txt --answer_file ref.txt ...
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from epfl_megatron_amd import get_args  # noqa: E402
from epfl_megatron_amd.initialize import initialize_megatron  # noqa: E402


def get_tasks_args(parser):
    import finetune
    parser = finetune.extra_args(parser)
    g = parser.add_argument_group(title="tasks")
    g.add_argument("--task", type=str, required=True)
    g.add_argument("--sample_input_file", type=str, default=None)
    g.add_argument("--sample_output_file", type=str, default=None)
    g.add_argument("--prompt_file", type=str, default=None)
    g.add_argument("--prompt_type", type=str, default=None, choices=["knowledge", "response"])
    g.add_argument("--num_prompt_examples", type=int, default=10)
    g.add_argument("--guess_file", type=str, default=None)
    g.add_argument("--answer_file", type=str, default=None)
    g.add_argument("--out_seq_length", type=int, default=100)
    g.add_argument("--api_prompt", action="store_true")
    g.add_argument("--megatron_api_url", type=str, default=None)
    return parser


def main(argv=None):
    initialize_megatron(get_tasks_args, args_list=argv)
    args = get_args()
    if args.num_layers_per_virtual_pipeline_stage is not None:
        raise SystemExit("Interleaved pipeline schedule is not supported for downstream tasks.")
    if args.task == "MSDP-PROMPT":
        from tasks.msdp.prompt import main as run
    elif args.task == "MSDP-EVAL-F1":
        from tasks.msdp.evaluate import main as run
    else:
        raise NotImplementedError(f"Task {args.task} is not implemented.")
    return run()


if __name__ == "__main__":
    main()

"""Serve a checkpoint over REST (reference ``tools/run_text_generation_server.py``).

    torchrun --nproc_per_node N tools/run_text_generation_server.py \
        --model_name llama2 --load CKPT --use_checkpoint_args ... [--port 5000]

Rank 0 (first pipeline stage, TP rank 0) runs the HTTP server; all other
ranks wait in the command loop and join each generation collectively.
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), os.path.pardir)))

from epfl_megatron_amd import get_args, print_rank_0  # noqa: E402
from epfl_megatron_amd.checkpointing import load_checkpoint  # noqa: E402
from epfl_megatron_amd.initialize import initialize_megatron  # noqa: E402
from epfl_megatron_amd.models import (FalconModel, GPTModel, LlamaModel,  # noqa: E402
                                      ModelType)
from epfl_megatron_amd.training import get_model  # noqa: E402


def model_provider(pre_process=True, post_process=True):
    print_rank_0("building model ...")
    args = get_args()
    name = getattr(args, "model_name", "gpt")
    cls = {"gpt": GPTModel, "falcon": FalconModel, "llama": LlamaModel,
           "llama2": LlamaModel}[name]
    kw = {"version": 1 if name == "llama" else 2} if name in ("llama", "llama2") else {}
    return cls(num_tokentypes=0, parallel_output=False, pre_process=pre_process,
               post_process=post_process, **kw)


def add_text_generate_args(parser):
    g = parser.add_argument_group(title="text generation")
    g.add_argument("--temperature", type=float, default=1.0)
    g.add_argument("--top_p", type=float, default=0.0)
    g.add_argument("--top_k", type=int, default=0)
    g.add_argument("--out_seq_length", type=int, default=1024)
    g.add_argument("--model_name", choices={"gpt", "llama", "llama2", "falcon"}, default="gpt")
    g.add_argument("--port", type=int, default=5000)
    return parser


def main(argv=None):
    initialize_megatron(add_text_generate_args,
                        {"tokenizer_type": "GPT2BPETokenizer", "no_load_rng": True,
                         "no_load_optim": True}, args_list=argv)
    args = get_args()
    if args.num_layers_per_virtual_pipeline_stage is not None:
        print("Interleaved pipeline schedule is not yet supported for text generation.")
        return
    model = get_model(model_provider, ModelType.encoder_or_decoder, wrap_with_ddp=False)
    if args.load is not None:
        load_checkpoint(model, None, None)
    model = model[0]
    from epfl_megatron_amd.inference.server import MegatronServer, worker_loop
    import torch.distributed as dist
    if dist.get_rank() == 0:
        MegatronServer(model).run("0.0.0.0", args.port)
    else:
        worker_loop(model)


if __name__ == "__main__":
    main()

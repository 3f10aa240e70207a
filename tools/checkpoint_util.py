"""Re-shard a Megatron checkpoint to another TP x PP layout (reference
``tools/checkpoint_util.py`` + ``checkpoint_loader_megatron.py`` +
``checkpoint_saver_megatron.py``).

Same CLI::

    python tools/checkpoint_util.py --model_type llama2 --load_dir IN --save_dir OUT \
        --target_tensor_parallel_size 2 --target_pipeline_parallel_size 2 \
        [--true_vocab_size N | --vocab_file tokenizer.model] [--bf16]

Design: the reference streamed tensors from a loader process to a saver
process through an ``mp.Queue`` (to bound memory).  Here the loader
memory-maps every shard (``torch.load(mmap=True)``), so the merged model is a
set of views into page-cache-backed files and the saver slices it directly
in one process — same bounded memory, no serialisation round trip.  Loader /
saver plugins are still selected by ``--loader`` / ``--saver`` (modules named
``checkpoint_{loader,saver}_<name>`` exposing ``add_arguments`` and
``load_checkpoint(args) -> (metadata, full)`` / ``save_checkpoint(args, metadata, full)``).
"""
import argparse
import importlib
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), os.path.pardir)))
sys.path.insert(0, os.path.abspath(os.path.dirname(__file__)))


def load_plugin(plugin_type, name):
    for module_name in (f"checkpoint_{plugin_type}_{name}", name):
        try:
            plugin = importlib.import_module(module_name)
            break
        except ModuleNotFoundError:
            continue
    else:
        sys.exit(f"Unable to load {plugin_type} plugin {name}. Exiting.")
    if not hasattr(plugin, "add_arguments"):
        sys.exit(f"{module_name} module is not a plugin. Exiting.")
    print(f"Loaded {module_name} as the {plugin_type}.")
    return plugin


def main(argv=None):
    parser = argparse.ArgumentParser(description="Megatron Checkpoint Utility Arguments",
                                     allow_abbrev=False, conflict_handler="resolve")
    parser.add_argument("--model_type", type=str, required=True,
                        choices=["GPT", "BERT", "falcon", "llama", "llama2", "codellama"])
    parser.add_argument("--loader", type=str, default="megatron")
    parser.add_argument("--saver", type=str, default="megatron")
    parser.add_argument("--load_dir", type=str, required=True)
    parser.add_argument("--save_dir", type=str, required=True)
    parser.add_argument("--max_queue_size", type=int, default=50,
                        help="(kept for CLI compatibility; no queue is used)")
    parser.add_argument("--no_checking", action="store_false", dest="checking")
    parser.add_argument("--bf16", action="store_true", help="force bfloat16 weights")
    known, _ = parser.parse_known_args(argv)
    loader = load_plugin("loader", known.loader)
    saver = load_plugin("saver", known.saver)
    loader.add_arguments(parser)
    saver.add_arguments(parser)
    args = parser.parse_args(argv)
    md, full = loader.load_checkpoint(args)
    saver.save_checkpoint(args, md, full)
    print("Done")


if __name__ == "__main__":
    main()

"""Export (and optionally publish) a Hugging Face-format checkpoint
(reference ``tools/push_to_hub.py``).

    python tools/push_to_hub.py HF_DIR --output_folder OUT [--dtype bf16] \
        [--rope_scaling_type linear --rope_scaling_factor 2.0] [--max_shard_size 10GB]
    python tools/push_to_hub.py HF_DIR --hf_repo_name org/name --auth_token ...

Typical flow: ``weights2megatron/megatron2hf.py`` -> this tool.  Converting
the dtype / RoPE-scaling config and writing ``--output_folder`` is local;
``--hf_repo_name`` uploads to the Hub (needs network access and a token; it
is never attempted implicitly).  The model directory is read locally only.
"""
import argparse
import sys

import torch

_DTYPES = {"fp16": torch.float16, "float16": torch.float16, "fp32": torch.float32,
           "float32": torch.float32, "bf16": torch.bfloat16, "bfloat16": torch.bfloat16,
           "auto": None}


def parse_args(argv=None):
    p = argparse.ArgumentParser(
        description="Push checkpoints in HF transformers format to the Huggingface Hub.")
    p.add_argument("model_name", type=str, help="path to a local HF model directory")
    p.add_argument("--dtype", type=str, default="auto", help="auto, bf16, fp16 or fp32")
    p.add_argument("--hf_repo_name", type=str, help="Hub repository to push to")
    p.add_argument("--auth_token", type=str, help="Hub access token")
    p.add_argument("--output_folder", type=str, help="write the (converted) model here")
    p.add_argument("--max_shard_size", type=str, default="10GB")
    p.add_argument("--unsafe", action="store_true", help="disable safetensors serialization")
    p.add_argument("--rope_scaling_type", type=str, default="linear")
    p.add_argument("--rope_scaling_factor", type=float)
    p.add_argument("--trust_remote_code", action="store_true")
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    if args.dtype not in _DTYPES:
        print(f"Unsupported dtype: {args.dtype}")
        sys.exit(1)
    if not args.hf_repo_name and not args.output_folder:
        print("Please specify either `--hf_repo_name` to push to HF or `--output_folder` to "
              "export the model to a local folder.")
        sys.exit(1)
    from transformers import AutoModelForCausalLM, AutoTokenizer
    tokenizer = None
    try:
        tokenizer = AutoTokenizer.from_pretrained(args.model_name)
        print(f"Tokenizer: {type(tokenizer).__name__} (vocab_size: {len(tokenizer):,})")
        for tok in tokenizer.all_special_tokens:
            print(f"{tok}: {tokenizer.convert_tokens_to_ids(tok)}")
    except (OSError, ValueError) as e:
        print(f"no tokenizer exported with the model ({e}); continuing with weights only")
    model = AutoModelForCausalLM.from_pretrained(args.model_name, torch_dtype=_DTYPES[args.dtype],
                                                 trust_remote_code=args.trust_remote_code)
    print(f"Model: {type(model).__name__} (num_parameters={model.num_parameters():,})")
    if args.rope_scaling_type is not None and args.rope_scaling_factor is not None:
        if args.rope_scaling_type not in ("linear", "dynamic") or args.rope_scaling_factor < 1.0:
            raise ValueError("rope scaling: type linear|dynamic and factor >= 1.0")
        scaling = {"type": args.rope_scaling_type, "rope_type": args.rope_scaling_type,
                   "factor": args.rope_scaling_factor}
        print(f"Setting rope_scaling {scaling} (old: {getattr(model.config, 'rope_scaling', None)})")
        model.config.rope_scaling = scaling
    safe = not args.unsafe
    if args.output_folder:
        model.save_pretrained(args.output_folder, max_shard_size=args.max_shard_size,
                              safe_serialization=safe)
        if tokenizer is not None:
            tokenizer.save_pretrained(args.output_folder)
        print(f"saved to {args.output_folder}")
    if args.hf_repo_name:
        print(f"pushing to the Hub as {args.hf_repo_name} ...")
        model.push_to_hub(args.hf_repo_name, token=args.auth_token,
                          max_shard_size=args.max_shard_size, safe_serialization=safe)
        if tokenizer is not None:
            tokenizer.push_to_hub(args.hf_repo_name, token=args.auth_token)


if __name__ == "__main__":
    main()

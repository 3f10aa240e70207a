"""Command-line flag system.

Same public CLI as the reference (underscore-style flags, identical names,
defaults and derived fields; see reference ``megatron/arguments.py:14-1073``),
but expressed declaratively: every flag is one row of a table, grouped by
section, and the parser is generated from the table.  ``validate_args``
reproduces the reference's derivations (``megatron/arguments.py:52-345``)
plus MI355X-specific additions (bucket sizes, synthetic data, kernel knobs).
"""

import argparse
import warnings
import os

import torch

from ..models.enums import PositionEmbeddingType

_T = True
_F = False


def _flag(name, **kw):
    return (name, kw)


def _pos_emb_type(x):
    if isinstance(x, PositionEmbeddingType):
        return x
    return PositionEmbeddingType[x]


# ---------------------------------------------------------------------------
# Flag table.  Each section -> list of (flag, argparse-kwargs).
# ---------------------------------------------------------------------------
FLAG_TABLE = {
    "Transformer-Engine": [
        _flag("--fp8_e4m3", action="store_true"),
        _flag("--fp8_hybrid", action="store_true"),
        _flag("--no_fp8_wgrad", action="store_false", dest="fp8_wgrad"),
        _flag("--fp8_margin", type=int, default=0),
        _flag("--fp8_interval", type=int, default=1),
        _flag("--transformer_impl", default="local", choices=["local", "transformer_engine"]),
        _flag("--fp8_amax_history_len", type=int, default=1),
        _flag("--fp8_amax_compute_algo", default="most_recent", choices=["most_recent", "max"]),
    ],
    "inference": [
        _flag("--inference_batch_times_seqlen_threshold", type=int, default=512),
        _flag("--max_tokens_to_oom", type=int, default=12000),
        _flag("--inference_hip_graph", action="store_true",
              help="replay single-token decode forwards from a captured hipGraph "
                   "(any TP / PP size: under PP every stage replays its own graph between an "
                   "eager receive and send; the whole-loop greedy decoder needs PP = 1; "
                   "inference/hip_graph.py)"),
    ],
    "network size": [
        _flag("--num_layers", type=int, default=None),
        _flag("--encoder_num_layers", type=int, default=None),
        _flag("--decoder_num_layers", type=int, default=None),
        _flag("--hidden_size", type=int, default=None),
        _flag("--ffn_hidden_size", type=int, default=None),
        _flag("--num_attention_heads", type=int, default=None),
        _flag("--num_attention_heads_kv", type=int, default=None),
        _flag("--kv_channels", type=int, default=None),
        _flag("--max_position_embeddings", type=int, default=None),
        _flag("--make_vocab_size_divisible_by", type=int, default=128),
        _flag("--layernorm_epsilon", type=float, default=1e-5),
        _flag("--apply_residual_connection_post_layernorm", action="store_true"),
        _flag("--use_bias", action="store_true"),
        _flag("--use_rms_norm", action="store_true"),
        _flag("--use_post_ln", action="store_true"),
        _flag("--onnx_safe", type=bool, required=False),
        _flag("--glu_activation", type=str, default=None,
              choices=["geglu", "liglu", "reglu", "swiglu"]),
        _flag("--position_embedding_type", type=_pos_emb_type,
              default=PositionEmbeddingType.absolute,
              choices=list(PositionEmbeddingType)),
        _flag("--rope_scaling_factor", type=float, default=1.0),
        _flag("--parallel_attn", action="store_true"),
        _flag("--parallel_layernorm", action="store_true"),
        _flag("--no_tie_embed_logits", action="store_false", dest="tie_embed_logits"),
    ],
    "logging": [
        _flag("--log_params_norm", action="store_true"),
        _flag("--log_num_zeros_in_grad", action="store_true"),
        _flag("--timing_log_level", type=int, default=0, choices=range(0, 3)),
        # reference spelling (megatron/arguments.py:492, store_false: passing it
        # turns the level-1 timer barriers OFF); the descriptive name is an alias
        _flag(("--barrier_with_L1_time", "--no_barrier_with_level_1_timing"),
              action="store_false", dest="barrier_with_L1_time"),
        _flag("--timing_log_option", type=str, default="minmax",
              choices=["max", "minmax", "all"]),
        _flag("--tensorboard_log_interval", type=int, default=1),
        _flag("--tensorboard_queue_size", type=int, default=1000),
        _flag("--log_timers_to_tensorboard", action="store_true"),
        _flag("--log_batch_size_to_tensorboard", action="store_true"),
        _flag("--no_log_learnig_rate_to_tensorboard", action="store_false",
              dest="log_learning_rate_to_tensorboard_core"),
        _flag("--no_log_loss_scale_to_tensorboard", action="store_false",
              dest="log_loss_scale_to_tensorboard_core"),
        _flag("--log_validation_ppl_to_tensorboard", action="store_true"),
        _flag("--log_memory_to_tensorboard", action="store_true"),
        _flag("--log_world_size_to_tensorboard", action="store_true"),
        _flag("--wandb_logger", action="store_true"),
        _flag("--wandb_project", type=str, default=None),
        _flag("--wandb_entity", type=str, default="meditron"),
        _flag("--wandb_id", type=str, default=None),
        _flag("--wandb_resume", action="store_true"),
        _flag("--wandb_api_key", type=str, default=None),
        # MI355X additions: throughput / MFU in the log line.
        _flag("--log_throughput", action="store_true", default=True),
        _flag("--peak_tflops", type=float, default=2500.0,
              help="dense bf16 peak per GPU used as the MFU denominator"),
    ],
    "regularization": [
        _flag("--attention_dropout", type=float, default=0.1),
        _flag("--hidden_dropout", type=float, default=0.1),
        _flag("--lima_dropout", action="store_true"),
        _flag("--weight_decay", type=float, default=0.01),
        _flag("--start_weight_decay", type=float, default=None),
        _flag("--end_weight_decay", type=float, default=None),
        _flag("--weight_decay_incr_style", type=str, default="constant",
              choices=["constant", "linear", "cosine"]),
        _flag("--clip_grad", type=float, default=1.0),
        _flag("--adam_beta1", type=float, default=0.9),
        _flag("--adam_beta2", type=float, default=0.999),
        _flag("--adam_eps", type=float, default=1e-08),
        _flag("--sgd_momentum", type=float, default=0.9),
    ],
    "training": [
        _flag("--micro_batch_size", type=int, default=None),
        _flag("--batch_size", type=int, default=None),
        _flag("--global_batch_size", type=int, default=None),
        _flag("--rampup_batch_size", nargs="*", default=None),
        _flag("--recompute_activations", action="store_true"),
        _flag("--recompute_granularity", type=str, default=None, choices=["full", "selective"]),
        _flag("--distribute_saved_activations", action="store_true"),
        _flag("--recompute_method", type=str, default=None, choices=["uniform", "block"]),
        _flag("--recompute_num_layers", type=int, default=1),
        _flag("--recompute_memory_budget_gb", type=float, default=None,
              help="MI355X: recompute (block method) only as many layers per pipeline "
                   "stage as needed for the estimated per-GPU peak to fit this many GB "
                   "(utils/memory_model.py); 0 recomputed layers disables recompute"),
        _flag("--train_iters", type=int, default=None),
        _flag("--train_samples", type=int, default=None),
        _flag("--log_interval", type=int, default=100),
        _flag("--exit_interval", type=int, default=None),
        _flag("--exit_duration_in_mins", type=int, default=None),
        _flag("--exit_signal_handler", action="store_true"),
        _flag("--tensorboard_dir", type=str, default=None),
        _flag("--no_masked_softmax_fusion", action="store_false", dest="masked_softmax_fusion"),
        _flag("--no_bias_gelu_fusion", action="store_false", dest="bias_gelu_fusion"),
        _flag("--no_bias_dropout_fusion", action="store_false", dest="bias_dropout_fusion"),
        _flag("--use_flash_attn", action="store_true"),
        _flag("--optimizer", type=str, default="adam", choices=["adam", "sgd"]),
        _flag("--dataloader_type", type=str, default=None, choices=["single", "cyclic"]),
        _flag("--no_async_tensor_model_parallel_allreduce", action="store_false",
              dest="async_tensor_model_parallel_allreduce"),
        _flag("--no_persist_layer_norm", action="store_true"),
        _flag("--sequence_parallel", action="store_true"),
        _flag("--no_gradient_accumulation_fusion", action="store_false",
              dest="gradient_accumulation_fusion"),
    ],
    "initialization": [
        _flag("--seed", type=int, default=1234),
        _flag("--data_parallel_random_init", action="store_true"),
        _flag("--init_method_std", type=float, default=0.02),
        _flag("--init_method_xavier_uniform", action="store_true"),
    ],
    "learning rate": [
        _flag("--lr", type=float, default=None),
        _flag("--lr_decay_style", type=str, default="linear",
              choices=["constant", "linear", "cosine", "inverse-square-root"]),
        _flag("--lr_decay_iters", type=int, default=None),
        _flag("--lr_decay_samples", type=int, default=None),
        _flag("--lr_warmup_fraction", type=float, default=None),
        _flag("--lr_warmup_iters", type=int, default=0),
        _flag("--lr_warmup_samples", type=int, default=0),
        _flag("--min_lr", type=float, default=0.0),
        _flag("--override_opt_param_scheduler", action="store_true"),
        _flag("--use_checkpoint_opt_param_scheduler", action="store_true"),
    ],
    "checkpointing": [
        _flag("--save", type=str, default=None),
        _flag("--save_interval", type=int, default=None),
        _flag("--no_save_optim", action="store_true", default=None),
        _flag("--no_save_rng", action="store_true", default=None),
        _flag("--load", type=str, default=None),
        _flag("--no_load_optim", action="store_true", default=None),
        _flag("--no_load_rng", action="store_true", default=None),
        _flag("--finetune", action="store_true"),
        _flag("--no_initialization", action="store_false", dest="perform_initialization"),
        _flag("--use_checkpoint_args", action="store_true"),
        _flag("--async_save", action="store_true",
              help="MI355X addition: stage tensors to host and write on a background thread"),
    ],
    "mixed precision": [
        _flag("--fp16", action="store_true"),
        _flag("--bf16", action="store_true"),
        _flag("--loss_scale", type=float, default=None),
        _flag("--initial_loss_scale", type=float, default=2 ** 32),
        _flag("--min_loss_scale", type=float, default=1.0),
        _flag("--loss_scale_window", type=float, default=1000),
        _flag("--hysteresis", type=int, default=2),
        _flag("--fp32_residual_connection", action="store_true"),
        _flag("--no_query_key_layer_scaling", action="store_false",
              dest="apply_query_key_layer_scaling"),
        _flag("--attention_softmax_in_fp32", action="store_true"),
        _flag("--accumulate_allreduce_grads_in_fp32", action="store_true"),
        _flag("--fp16_lm_cross_entropy", action="store_true"),
    ],
    "distributed": [
        _flag("--tensor_model_parallel_size", type=int, default=1),
        _flag("--pipeline_model_parallel_size", type=int, default=1),
        _flag("--pipeline_model_parallel_split_rank", type=int, default=None),
        _flag("--context_parallel_size", type=int, default=1,
              help="MI355X addition: split every sequence over this many consecutive DP "
                   "ranks; attention runs as a ring over them (parallel/context.py)"),
        _flag("--num_layers_per_virtual_pipeline_stage", type=int, default=None),
        _flag("--distributed_backend", default="nccl", choices=["nccl", "gloo"]),
        _flag("--DDP_impl", default="local", choices=["local", "torch"]),
        _flag("--no_contiguous_buffers_in_local_ddp", action="store_false",
              dest="use_contiguous_buffers_in_local_ddp"),
        _flag("--no_scatter_gather_tensors_in_pipeline", action="store_false",
              dest="scatter_gather_tensors_in_pipeline"),
        _flag("--use_ring_exchange_p2p", action="store_true", default=False),
        _flag("--local_rank", type=int, default=None),
        _flag("--use_cpu_initialization", action="store_true", default=None),
        _flag("--empty_unused_memory_level", default=0, type=int, choices=[0, 1, 2]),
        _flag("--standalone_embedding_stage", action="store_true", default=False),
        _flag("--use_distributed_optimizer", action="store_true"),
        # MI355X additions: bucketed, overlapped DP reduction sized for xGMI.
        _flag("--ddp_bucket_size_mb", type=float, default=256.0,
              help="fp32 gradient bucket size (MiB) for the overlapped DP reduction"),
        _flag("--simulated_tensor_parallel_size", type=int, default=None,
              help="MI355X per-rank proxy: build and run ONE tensor-parallel rank of a "
                   "TP=N model in this process (sharded weights, heads, vocab and, with "
                   "--sequence_parallel, s/N-row norms / residuals / dropout). TP "
                   "collectives become local loopbacks (all-gather writes the shard into "
                   "every rank's slot, reduce-scatter keeps this rank's own chunk without "
                   "reducing, all-reduce / broadcast are identities) that are accounted in "
                   "the comm table with the bytes a real rank would send"),
        _flag("--ddp_comm_groups", type=int, default=1,
              help="communicators over the DP ranks; DDP buckets are issued round-robin "
                   "on them so several reduce concurrently (one RCCL stream each)"),
        _flag("--tp_xgmi_allreduce_kb", type=int, default=0,
              help="route tensor-parallel sum all-reduces and all-gathers of at most this "
                   "many KiB per rank (contiguous, 16-B sized) through the one-shot xGMI "
                   "peer-memory kernel (parallel/xgmi.py) instead of RCCL; 0 = off.  For the "
                   "latency-bound [b, h] all-reduces and logits all-gathers of TP decode"),
        _flag("--tp_xgmi_allgather_kb", type=int, default=None,
              help="per-rank cap (KiB) of the tensor-parallel all-gathers routed through the "
                   "one-shot xGMI kernel (default: --tp_xgmi_allreduce_kb).  Sized for the "
                   "sequence-parallel [s/tp, b, h] pieces (multi-MiB) it lets the all-gather "
                   "take the W-1 links at once instead of an RCCL ring"),
        _flag("--tp_xgmi_timeout_ms", type=int, default=None,
              help="wall-clock bound (ms) of a one-shot xGMI collective's wait on a peer "
                   "(default 60000, or EMA_XGMI_TIMEOUT_MS): long, so a late but healthy "
                   "rank never trips it; a timed-out wait NaN-fills the output, skips the "
                   "optimizer step on every rank and raises at the next log / checkpoint"),
        _flag("--sp_regather_inputs", action="store_true",
              help="sequence parallel: all-gather the inputs of the column-parallel products "
                   "(QKV, fc1, LM head) again in the backward for their weight gradients, as "
                   "the reference does, instead of keeping the forward's gathered copies "
                   "(default: kept; 2 fewer full-size TP collectives per layer and "
                   "micro-batch for [s, b, h] of HBM per product)"),
        _flag("--no_overlap_grad_reduce", action="store_false", dest="overlap_grad_reduce"),
        _flag("--no_overlap_param_gather", action="store_false", dest="overlap_param_gather",
              help="dist-opt: all-gather parameters synchronously at step end instead of "
                   "overlapping the gather with the next forward"),
        _flag("--allow_interleaved_pp2", action="store_true",
              help="lift the reference's PP>2 restriction for the interleaved schedule"),
        _flag("--distributed_timeout_minutes", type=int, default=10),
        _flag("--no_comm_selfcheck", action="store_false", dest="comm_selfcheck",
              help="skip the startup check of the collectives on the real backend "
                   "(parallel/selfcheck.py)"),
    ],
    "validation": [
        _flag("--eval_iters", type=int, default=100),
        _flag("--eval_interval", type=int, default=1000),
    ],
    "data and dataloader": [
        _flag("--data_path", nargs="*", default=None),
        _flag("--split", type=str, default="969, 30, 1"),
        _flag("--train_data_path", nargs="*", default=None),
        _flag("--valid_data_path", nargs="*", default=None),
        _flag("--test_data_path", nargs="*", default=None),
        _flag("--vocab_file", type=str, default=None),
        _flag("--merge_file", type=str, default=None),
        _flag("--vocab_extra_ids", type=int, default=0),
        _flag("--vocab_extra_ids_list", type=str, default=None),
        _flag("--seq_length", type=int, default=None),
        _flag("--encoder_seq_length", type=int, default=None),
        _flag("--decoder_seq_length", type=int, default=None),
        _flag("--retriever_seq_length", type=int, default=256),
        _flag("--sample_rate", type=float, default=1.0),
        _flag("--mask_prob", type=float, default=0.15),
        # upstream Megatron flag the reference's pretrain_bert.py reads but never defines
        _flag("--bert_no_binary_head", action="store_false", dest="bert_binary_head"),
        _flag("--short_seq_prob", type=float, default=0.1),
        _flag("--mmap_warmup", action="store_true"),
        _flag("--num_workers", type=int, default=2),
        _flag("--tokenizer_type", type=str, default=None,
              choices=["BertWordPieceLowerCase", "BertWordPieceCase", "GPT2BPETokenizer",
                       "SentencePieceTokenizer", "FalconTokenizer", "NullTokenizer"]),
        _flag("--tokenizer_model", type=str, default=None),
        _flag("--no_new_tokens", action="store_false", dest="new_tokens"),
        _flag("--data_impl", type=str, default="infer", choices=["lazy", "cached", "mmap", "infer"]),
        _flag("--reset_position_ids", action="store_true"),
        _flag("--reset_attention_mask", action="store_true"),
        _flag("--eod_mask_loss", action="store_true"),
        # MI355X addition: synthetic data for benchmarks (no corpus needed).
        _flag("--synthetic_data", action="store_true"),
        _flag("--synthetic_vocab_size", type=int, default=32000),
        _flag("--synthetic_pattern", type=str, default="uniform", choices=["uniform", "cycle"],
              help="uniform: i.i.d. tokens; cycle: walk along a fixed random permutation "
                   "(learnable, same cost)"),
    ],
    "autoresume": [
        _flag("--adlr_autoresume", action="store_true"),
        _flag("--adlr_autoresume_interval", type=int, default=1000),
    ],
    "biencoder": [
        _flag("--ict_head_size", type=int, default=None),
        _flag("--biencoder_projection_dim", type=int, default=0),
        _flag("--biencoder_shared_query_context_model", action="store_true"),
        _flag("--ict_load", type=str, default=None),
        _flag("--bert_load", type=str, default=None),
        _flag("--titles_data_path", type=str, default=None),
        _flag("--query_in_block_prob", type=float, default=0.1),
        _flag("--use_one_sent_docs", action="store_true"),
        _flag("--evidence_data_path", type=str, default=None),
        _flag("--retriever_report_topk_accuracies", nargs="+", type=int, default=[]),
        _flag("--retriever_score_scaling", action="store_true"),
        _flag("--block_data_path", type=str, default=None),
        _flag("--embedding_path", type=str, default=None),
        _flag("--indexer_batch_size", type=int, default=128),
        _flag("--indexer_log_interval", type=int, default=1000),
    ],
    "vision": [
        _flag("--num_classes", type=int, default=1000),
        _flag("--img_h", type=int, default=224),
        _flag("--img_w", type=int, default=224),
        _flag("--num_channels", type=int, default=3),
        _flag("--patch_dim", type=int, default=16),
        _flag("--classes_fraction", type=float, default=1.0),
        _flag("--data_per_class_fraction", type=float, default=1.0),
        _flag("--no_data_sharding", action="store_false", dest="data_sharding"),
        _flag("--head_lr_mult", type=float, default=1.0),
        _flag("--iter_per_epoch", type=int, default=1250),
        _flag("--dino_local_img_size", type=int, default=96),
        _flag("--dino_local_crops_number", type=int, default=10),
        _flag("--dino_head_hidden_size", type=int, default=2048),
        _flag("--dino_bottleneck_size", type=int, default=256),
        _flag("--dino_freeze_last_layer", type=float, default=1),
        _flag("--dino_norm_last_layer", action="store_true"),
        _flag("--dino_warmup_teacher_temp", type=float, default=0.04),
        _flag("--dino_teacher_temp", type=float, default=0.07),
        _flag("--dino_warmup_teacher_temp_epochs", type=int, default=30),
    ],
}


def build_base_parser():
    parser = argparse.ArgumentParser(description="epfl_megatron_amd arguments",
                                     allow_abbrev=False)
    for section, flags in FLAG_TABLE.items():
        group = parser.add_argument_group(title=section)
        for name, kw in flags:
            names = name if isinstance(name, tuple) else (name,)
            group.add_argument(*names, **kw)
    return parser


def parse_args(extra_args_provider=None, args_list=None):
    """Parse flags; rank/world size come from the torchrun environment."""
    parser = build_base_parser()
    if extra_args_provider is not None:
        parser = extra_args_provider(parser)
    args = parser.parse_args(args_list)
    args.rank = int(os.getenv("RANK", "0"))
    args.world_size = int(os.getenv("WORLD_SIZE", "1"))
    return args


def _require(cond, msg):
    if not cond:
        raise AssertionError(msg)


def _log0(args, msg):
    if args.rank == 0:
        print(msg, flush=True)


def _derive_parallel_sizes(args):
    args.tensor_model_parallel_size = min(args.tensor_model_parallel_size, args.world_size)
    _require(args.world_size % args.tensor_model_parallel_size == 0,
             f"world size ({args.world_size}) is not divisible by tensor model parallel size "
             f"({args.tensor_model_parallel_size})")
    args.pipeline_model_parallel_size = min(
        args.pipeline_model_parallel_size, args.world_size // args.tensor_model_parallel_size)
    args.transformer_pipeline_model_parallel_size = (
        args.pipeline_model_parallel_size - 1 if args.standalone_embedding_stage
        else args.pipeline_model_parallel_size)
    mp = args.pipeline_model_parallel_size * args.tensor_model_parallel_size
    _require(args.world_size % mp == 0,
             f"world size is not divisible by tensor parallel size "
             f"({args.tensor_model_parallel_size}) times pipeline parallel size "
             f"({args.pipeline_model_parallel_size})")
    cp = getattr(args, "context_parallel_size", 1) or 1
    _require(args.world_size % (mp * cp) == 0,
             f"world size ({args.world_size}) is not divisible by tp x pp ({mp}) times "
             f"context parallel size ({cp})")
    # data_parallel_size counts the ranks that read DIFFERENT samples (batch
    # accounting); gradients are reduced over data_parallel_size x cp ranks.
    args.data_parallel_size = args.world_size // mp // cp
    _log0(args, f"using world size: {args.world_size}, data-parallel-size: "
                f"{args.data_parallel_size}, tensor-model-parallel size: "
                f"{args.tensor_model_parallel_size}, pipeline-model-parallel size: "
                f"{args.pipeline_model_parallel_size}, context-parallel size: {cp} ")
    if args.pipeline_model_parallel_size > 1 and args.pipeline_model_parallel_split_rank is not None:
        _require(args.pipeline_model_parallel_split_rank < args.pipeline_model_parallel_size,
                 "split rank needs to be less than pipeline model parallel size")


def _apply_defaults(args, defaults):
    for key, value in defaults.items():
        if getattr(args, key, None) is not None:
            _log0(args, f"WARNING: overriding default arguments for {key}:{value} "
                        f"with {key}:{getattr(args, key)}")
        else:
            setattr(args, key, value)


def _derive_batch_and_vpp(args):
    if getattr(args, "batch_size", None) is not None and args.micro_batch_size is None:
        args.micro_batch_size = args.batch_size
    _require(args.micro_batch_size is not None and args.micro_batch_size > 0,
             "micro_batch_size must be set and positive")
    if args.global_batch_size is None:
        args.global_batch_size = args.micro_batch_size * args.data_parallel_size
        _log0(args, f"setting global batch size to {args.global_batch_size}")
    _require(args.global_batch_size > 0, "global batch size must be positive")
    if args.num_layers_per_virtual_pipeline_stage is not None:
        # Reference requires PP > 2 (megatron/arguments.py:117-120).  The schedule
        # math is valid at PP == 2 as well; --allow_interleaved_pp2 lifts it.
        min_pp = 2 if args.allow_interleaved_pp2 else 3
        _require(args.pipeline_model_parallel_size >= min_pp,
                 "pipeline-model-parallel size should be greater than 2 with interleaved "
                 "schedule (pass --allow_interleaved_pp2 to permit PP=2)")
        _require(args.num_layers % args.num_layers_per_virtual_pipeline_stage == 0,
                 "number of layers is not divisible by number of layers per virtual "
                 "pipeline stage")
        args.virtual_pipeline_model_parallel_size = (
            (args.num_layers // args.transformer_pipeline_model_parallel_size)
            // args.num_layers_per_virtual_pipeline_stage)
    else:
        args.virtual_pipeline_model_parallel_size = None


def _derive_dtypes(args):
    args.params_dtype = torch.float
    if args.fp16:
        _require(not args.bf16, "fp16 and bf16 are exclusive")
        args.params_dtype = torch.half
    if args.bf16:
        _require(not args.fp16, "fp16 and bf16 are exclusive")
        args.params_dtype = torch.bfloat16
        if not args.accumulate_allreduce_grads_in_fp32:
            args.accumulate_allreduce_grads_in_fp32 = True
            _log0(args, "accumulate and all-reduce gradients in fp32 for bfloat16 data type.")
    _log0(args, f"using {args.params_dtype} for parameters ...")
    if args.accumulate_allreduce_grads_in_fp32 or args.use_distributed_optimizer:
        _require(args.DDP_impl == "local", "fp32 grad accumulation / dist-opt need local DDP")
        _require(args.use_contiguous_buffers_in_local_ddp,
                 "fp32 grad accumulation / dist-opt need contiguous buffers")
    if args.DDP_impl == "torch":
        args.use_contiguous_buffers_in_local_ddp = False


def _derive_schedule_and_model(args):
    if args.dataloader_type is None:
        args.dataloader_type = "single"
    args.consumed_train_samples = 0
    args.consumed_valid_samples = 0
    args.variable_seq_lengths = False
    if args.train_iters:
        _require(args.train_samples is None, "expected iteration-based training")
        _require(args.lr_decay_samples is None, "expected iteration-based learning rate decay")
        _require(args.lr_warmup_samples == 0, "expected iteration-based learning rate warmup")
        _require(args.rampup_batch_size is None,
                 "expected no batch-size rampup for iteration-based training")
        if args.lr_warmup_fraction is not None:
            _require(args.lr_warmup_iters == 0,
                     "can only specify one of lr_warmup_fraction and lr_warmup_iters")
    if args.train_samples:
        _require(args.train_iters is None, "expected sample-based training")
        _require(args.lr_decay_iters is None, "expected sample-based learning rate decay")
        _require(args.lr_warmup_iters == 0, "expected sample-based learning rate warmup")
        if args.lr_warmup_fraction is not None:
            _require(args.lr_warmup_samples == 0,
                     "can only specify one of lr_warmup_fraction and lr_warmup_samples")
    if args.num_layers is not None:
        _require(args.encoder_num_layers is None,
                 "cannot have both num_layers and encoder_num_layers specified")
        args.encoder_num_layers = args.num_layers
    else:
        _require(args.encoder_num_layers is not None,
                 "either num_layers or encoder_num_layers should be specified")
        args.num_layers = args.encoder_num_layers
    if args.decoder_num_layers is None:
        # (the reference leaves it None and T5 then fails to build its decoder)
        args.decoder_num_layers = args.num_layers
    for req in ("num_layers", "hidden_size", "num_attention_heads"):
        _require(getattr(args, req) is not None, f"{req} argument is None")
    if args.ffn_hidden_size is None:
        args.ffn_hidden_size = 4 * args.hidden_size
    if args.kv_channels is None:
        _require(args.hidden_size % args.num_attention_heads == 0,
                 "hidden_size must be divisible by num_attention_heads")
        args.kv_channels = args.hidden_size // args.num_attention_heads
    if args.num_attention_heads_kv is None:
        args.num_attention_heads_kv = args.num_attention_heads
    _require(args.num_attention_heads % args.num_attention_heads_kv == 0,
             "num_attention_heads must be a multiple of num_attention_heads_kv")
    if args.seq_length is not None:
        _require(args.encoder_seq_length is None, "seq_length and encoder_seq_length conflict")
        args.encoder_seq_length = args.seq_length
    else:
        _require(args.encoder_seq_length is not None, "seq_length must be set")
        args.seq_length = args.encoder_seq_length
    args.position_embedding_type = _pos_emb_type(args.position_embedding_type)
    _require(args.max_position_embeddings is not None, "max_position_embeddings must be set")
    if args.seq_length is not None:
        _require(args.max_position_embeddings >= args.seq_length,
                 "max_position_embeddings must be >= seq_length")
    if args.decoder_seq_length is not None:
        _require(args.max_position_embeddings >= args.decoder_seq_length,
                 "max_position_embeddings must be >= decoder_seq_length")
    _require(args.rope_scaling_factor >= 1, "rope_scaling_factor must be >= 1")
    if args.lr is not None:
        _require(args.min_lr <= args.lr, "min_lr must be <= lr")
    if args.save is not None:
        _require(args.save_interval is not None, "--save requires --save_interval")
    if args.fp16_lm_cross_entropy:
        _require(args.fp16, "lm cross entropy in fp16 only support in fp16 mode.")
    if args.fp32_residual_connection:
        _require(args.fp16 or args.bf16,
                 "residual connection in fp32 only supported when using fp16 or bf16.")
    if args.weight_decay_incr_style == "constant":
        _require(args.start_weight_decay is None and args.end_weight_decay is None,
                 "start/end weight decay only valid with a non-constant style")
        args.start_weight_decay = args.weight_decay
        args.end_weight_decay = args.weight_decay
    else:
        _require(args.start_weight_decay is not None and args.end_weight_decay is not None,
                 "non-constant weight decay needs start and end values")


def _derive_recompute_and_parallel_features(args):
    if getattr(args, "use_ring_exchange_p2p", False):
        warnings.warn("--use_ring_exchange_p2p is accepted for compatibility and ignored: "
                      "pipeline p2p always runs as batched isend/irecv over RCCL "
                      "(parallel/pipeline/p2p.py; torch.distributed has no ring_exchange)",
                      stacklevel=2)
    if args.distribute_saved_activations:
        _require(args.tensor_model_parallel_size > 1,
                 "can distribute recomputed activations only across tensor model parallel groups")
        _require(args.recompute_granularity == "full",
                 "distributed recompute activations is only application to full recompute granularity")
        _require(args.recompute_method is not None,
                 "for distributed recompute activations to work you need to use a recompute method")
    if args.fp8_e4m3 or args.fp8_hybrid:
        _require(args.transformer_impl == "transformer_engine",
                 "transformer-engine required for fp8 training and inference")
    _require(not (args.fp8_e4m3 and args.fp8_hybrid),
             "cannot train with both fp8 e4m3 and hybrid formatting")
    if args.transformer_impl != "local":
        raise AssertionError("--transformer_impl transformer_engine is not available: the "
                             "MI355X build uses its own fused HIP layer (local)")
    if args.recompute_granularity == "selective":
        _require(args.recompute_method is None,
                 "recompute method is not yet supported for selective recomputing granularity")
    if not args.parallel_attn:
        _require(not args.parallel_layernorm,
                 "parallel_layernorm only implemented with parallel_attention")
    sim_tp = getattr(args, "simulated_tensor_parallel_size", None)
    if sim_tp:
        _require(args.tensor_model_parallel_size == 1 and args.pipeline_model_parallel_size == 1
                 and args.world_size == 1,
                 "--simulated_tensor_parallel_size runs one rank of a TP model in a single "
                 "process (world size 1, no real TP / PP)")
    if args.tensor_model_parallel_size == 1 and not (sim_tp and sim_tp > 1):
        args.sequence_parallel = False
    if args.sequence_parallel:
        args.async_tensor_model_parallel_allreduce = False
    cp = getattr(args, "context_parallel_size", 1) or 1
    if cp > 1:
        _require(args.seq_length % (2 * cp) == 0,
                 f"seq_length ({args.seq_length}) is not divisible by 2 x context parallel "
                 f"size ({cp}) (zig-zag sequence split)")
        _require(not sim_tp, "--simulated_tensor_parallel_size excludes context parallelism")
        # the ring-attention pair kernels apply no attention dropout:
        # refuse a configuration whose CP=1 counterpart would drop attention probs
        _require(args.attention_dropout == 0 or args.use_flash_attn,
                 "context parallelism applies no attention dropout: set --attention_dropout 0 "
                 "(or --use_flash_attn, which has none either)")
    for flag in ("tp_xgmi_allreduce_kb", "tp_xgmi_allgather_kb"):
        xg = getattr(args, flag, 0) or 0
        _require(xg >= 0 and xg % 4 == 0 and xg <= 65536,
                 f"--{flag} must be a multiple of 4 in [0, 65536] "
                 "(the one-shot kernel moves 4 KiB per workgroup)")
    # Reference defect D17: the GQA view silently breaks when KV heads do not
    # split evenly over TP ranks; we check it explicitly.
    if args.num_attention_heads_kv % (sim_tp or args.tensor_model_parallel_size) != 0:
        raise AssertionError("num_attention_heads_kv must be divisible by "
                             "tensor_model_parallel_size")


def validate_args(args, defaults=None):
    """Derive and cross-check args (reference ``megatron/arguments.py:52-345``)."""
    defaults = defaults or {}
    _derive_parallel_sizes(args)
    if args.recompute_activations:
        args.recompute_granularity = "selective"
    del args.recompute_activations
    _apply_defaults(args, defaults)
    _derive_batch_and_vpp(args)
    _derive_dtypes(args)
    _derive_schedule_and_model(args)
    _derive_recompute_and_parallel_features(args)
    if getattr(args, "log_learning_rate_to_tensorboard", None) is None:
        args.log_learning_rate_to_tensorboard = args.log_learning_rate_to_tensorboard_core
    if getattr(args, "log_loss_scale_to_tensorboard", None) is None:
        args.log_loss_scale_to_tensorboard = args.log_loss_scale_to_tensorboard_core
    print_args(args)
    return args


def print_args(args):
    if args.rank != 0:
        return
    print("------------------------ arguments ------------------------", flush=True)
    lines = [f"  {k} {'.' * (48 - len(k))} {v}" for k, v in vars(args).items()]
    for line in sorted(lines, key=str.lower):
        print(line, flush=True)
    print("-------------------- end of arguments ---------------------", flush=True)

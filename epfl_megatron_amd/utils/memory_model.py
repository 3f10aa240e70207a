"""Per-GPU memory model and the budget-driven recompute policy.

MI355X has 288 GB of HBM3E per GPU, so the right amount of activation
recompute is usually far less than the reference's "recompute everything"
setting for its large-model configurations (``megatron/arguments.py:287-318``,
``megatron/model/transformer.py:1079-1145``).  ``--recompute_memory_budget_gb
B`` asks for the smallest number of recomputed layers (``block`` method: the
first N layers of each pipeline chunk keep only their input) whose estimated
peak fits in B GB; 0 means no recompute at all.

The estimate counts, per GPU:
* static state: bf16 weights, fp32 ``main_grad``, fp32 master + Adam moments
  (divided over DP with the distributed optimizer), and the per-step bf16 W^T
  cache of the dgrad GEMMs;
* per layer and in-flight micro-batch, the tensors the forward saves for the
  backward (GLU MLP, fused residual norms, FlashAttention), with s/tp-row
  residual-stream tensors under sequence parallelism, plus the full-sequence
  QKV / fc1 inputs the SP forward keeps for the wgrads (unless
  ``--sp_regather_inputs``);
* a recomputed layer keeps only its input; one layer's activations are live
  again while it is recomputed;
* the LM-head logits and loss workspace, and a fixed allowance for GEMM /
  collective workspaces and allocator fragmentation.

It is a model, not a measurement: ``bench.py`` reports the real peak
(``max_mem_gb``) next to the estimate.
"""
import math

GB = 1e9


def _tp(args):
    return getattr(args, "simulated_tensor_parallel_size", None) or args.tensor_model_parallel_size


def layer_activation_bytes(args, micro_batch=None):
    """Bytes one transformer layer saves for the backward, per micro-batch."""
    s = args.seq_length // (getattr(args, "context_parallel_size", 1) or 1)
    b = micro_batch or args.micro_batch_size
    tp = _tp(args)
    h = args.hidden_size
    hd = args.kv_channels or h // args.num_attention_heads
    nq = args.num_attention_heads
    nkv = args.num_attention_heads_kv or nq
    f = args.ffn_hidden_size or 4 * h
    t = s * b                                   # token rows through the GEMMs
    t_res = t // tp if args.sequence_parallel else t  # residual-stream rows
    el = 2 if (args.bf16 or args.fp16) else 4
    glu = 2 if args.glu_activation else 1
    n = 0
    n += 4 * t_res * h                          # norm inputs / GEMM inputs
    if args.sequence_parallel and tp > 1 and not getattr(args, "sp_regather_inputs", False):
        # the gathered [s, b, h] inputs of QKV and fc1, kept for their wgrads
        # instead of re-gathered (parallel/tensor/layers.py sp_keep_gathered);
        # they replace the saved s/tp-row GEMM inputs
        n += 2 * (t - t_res) * h
    n += t * (nq + 2 * nkv) * hd // tp          # fused QKV output (RoPE'd, read by FA backward)
    n += t * nq * hd // tp                      # attention output (+ o-proj input)
    n += t * glu * f // tp + (t * f // tp if glu == 2 else 0)  # fc1 pre-activation (+ GLU output)
    act = n * el + t * (nq // tp) * 4           # + FlashAttention log-sum-exp (fp32)
    if args.hidden_dropout > 0:
        act += 2 * t_res * h                    # dropout masks are regenerated: only a seed
    return act


def static_bytes(args, n_params_rank):
    """Weights, gradients, optimizer state and the W^T cache of one GPU."""
    el = 2 if (args.bf16 or args.fp16) else 4
    dp = args.data_parallel_size * (getattr(args, "context_parallel_size", 1) or 1) \
        if args.use_distributed_optimizer else 1
    weights = n_params_rank * el
    grads = n_params_rank * 4 if args.accumulate_allreduce_grads_in_fp32 or el == 2 else 0
    master = n_params_rank * 4 / dp if el == 2 else 0
    moments = 2 * n_params_rank * 4 / dp
    wt_cache = n_params_rank * el if el == 2 else 0
    return weights + grads + master + moments + wt_cache


def estimate(args, n_params_rank, layers, recomputed, in_flight=1):
    """Estimated peak bytes with ``recomputed`` of ``layers`` layers (per
    pipeline stage) recomputed and ``in_flight`` micro-batches live."""
    act = layer_activation_bytes(args)
    tp = _tp(args)
    t = args.seq_length // (getattr(args, "context_parallel_size", 1) or 1) * args.micro_batch_size
    t_res = t // tp if args.sequence_parallel else t
    inp = t_res * args.hidden_size * (2 if (args.bf16 or args.fp16) else 4)
    per_mb = (layers - recomputed) * act + recomputed * inp
    transient = act if recomputed else 0        # a layer being recomputed
    vocab = getattr(args, "padded_vocab_size", None) or 0
    logits = t * vocab // tp * 4 * 2            # fp32 logits + their gradient
    if args.sequence_parallel and tp > 1 and not getattr(args, "sp_regather_inputs", False):
        logits += (t - t_res) * args.hidden_size * 2 * in_flight  # LM-head input kept gathered
    workspace = 8 * GB
    return static_bytes(args, n_params_rank) + in_flight * per_mb + transient + logits + workspace


def auto_recompute_layers(args, n_params_rank, layers, budget_gb, in_flight=1):
    """Smallest number of recomputed layers that fits ``budget_gb`` (layers if none fits)."""
    for n in range(layers + 1):
        if estimate(args, n_params_rank, layers, n, in_flight) <= budget_gb * GB:
            return n
    return layers


def params_per_rank(args):
    """Parameters of one (TP, PP) rank, from the architecture (no model needed)."""
    from .flops import non_embedding_params
    tp = _tp(args)
    pp = args.pipeline_model_parallel_size
    total = non_embedding_params(args)
    vocab = getattr(args, "padded_vocab_size", None) or 0
    if getattr(args, "tie_embed_logits", False) is False:
        total += vocab * args.hidden_size       # input embedding (the head is counted above)
    return int(math.ceil(total / tp / pp))

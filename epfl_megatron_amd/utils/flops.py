"""Model FLOPs accounting for the throughput / MFU log (BASELINE.md formula).

``FLOPs/token = 6 * N_nonembedding + 12 * L * h * s`` (forward + backward, no
recompute credit), with N_nonembedding = every weight that takes part in a
GEMM: transformer layers plus the LM head (the input embedding lookup is not
a GEMM).  For Llama-2-7B this gives N = 6.61e9 as in BASELINE P1''.
"""


def non_embedding_params(args):
    h, L = args.hidden_size, args.num_layers
    hd = args.kv_channels or h // args.num_attention_heads
    nq, nkv = args.num_attention_heads, args.num_attention_heads_kv or args.num_attention_heads
    f = args.ffn_hidden_size or 4 * h
    v = getattr(args, "padded_vocab_size", None) or 0
    b = 1 if args.use_bias else 0
    qkv = h * hd * (nq + 2 * nkv) + b * hd * (nq + 2 * nkv)
    dense = hd * nq * h + b * h
    fc1 = h * f * (2 if args.glu_activation else 1) + b * f * (2 if args.glu_activation else 1)
    fc2 = f * h + b * h
    norms = (1 if args.parallel_attn and not args.parallel_layernorm else 2) * h * (1 if args.use_rms_norm else 2)
    per_layer = qkv + dense + fc1 + fc2 + norms
    return L * per_layer + v * h + h


def flops_per_token(args, seq_length=None):
    s = seq_length or args.seq_length
    # attention score/context GEMMs: 12 * L * (nq * hd) * s  (= 12 L h s unless
    # --kv_channels decouples the projection width from h, e.g. the TP proxies)
    hd = args.kv_channels or args.hidden_size // args.num_attention_heads
    proj = hd * args.num_attention_heads
    return 6.0 * non_embedding_params(args) + 12.0 * args.num_layers * proj * s

"""TP / SP / PP / interleaved-PP / DP / dist-opt runs == the single-process run.

The reference could only test parallelism on a real 8-GPU NCCL node; here every
layout of the tiny GPT / Llama models runs on CPU/gloo and must reproduce the
TP=PP=DP=1 loss trajectory (3 optimizer steps, identical weights and data).
"""
import hashlib

import pytest
import torch

from dist_utils import run_dist, init_framework, TINY_LLAMA, TINY_GPT


def _seed_of(name):
    return int(hashlib.md5(name.encode()).hexdigest()[:8], 16)


def _deterministic_init(model_chunks, args):
    """Fill every parameter from its GLOBAL name, then keep this rank's TP shard."""
    from epfl_megatron_amd.parallel import state
    from epfl_megatron_amd.utils.misc import unwrap_model
    tp = state.get_tensor_model_parallel_world_size()
    rank = state.get_tensor_model_parallel_rank()
    for chunk in unwrap_model(model_chunks):
        layer_of = {}
        for mname, mod in chunk.named_modules():
            if hasattr(mod, "layer_number") and mname.split(".")[-2:-1] == ["layers"]:
                layer_of[mname + "."] = mname.rsplit(".", 1)[0] + f".{mod.layer_number - 1}."
        for name, p in chunk.named_parameters():
            gname = name
            for local, glob in layer_of.items():
                if gname.startswith(local):
                    gname = glob + gname[len(local):]
                    break
            if gname == "word_embeddings.weight":  # last-stage copy of a tied embedding
                gname = "language_model.embedding.word_embeddings.weight"
            gname = gname.replace("module.", "")
            g = torch.Generator().manual_seed(_seed_of(gname))
            shape = list(p.shape)
            pdim = p.partition_dim if getattr(p, "tensor_model_parallel", False) else None
            if pdim is not None and tp > 1:
                shape[pdim] *= tp
            if len(shape) == 1 and not p.tensor_model_parallel:
                full = 1.0 + 0.1 * torch.randn(shape, generator=g)
            else:
                full = 0.05 * torch.randn(shape, generator=g)
            if pdim is not None and tp > 1:
                if "dense_h_to_4h" in gname and args.glu_activation:
                    up, gate = full.chunk(2, dim=0)
                    full = torch.cat([up.chunk(tp, 0)[rank], gate.chunk(tp, 0)[rank]], 0)
                else:
                    full = full.chunk(tp, dim=pdim)[rank]
            with torch.no_grad():
                p.copy_(full.to(p.dtype))


def _train(rank, world, argv, steps):
    import finetune
    init_framework(argv, finetune.extra_args)
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.optim import get_megatron_optimizer
    from epfl_megatron_amd.parallel import state
    from epfl_megatron_amd.training import (get_model, _get_optimizer_param_scheduler,
                                            build_train_valid_test_data_iterators, train_step)
    args = get_args()
    model = get_model(finetune.model_provider, ModelType.encoder_or_decoder)
    _deterministic_init(model, args)
    opt = get_megatron_optimizer(model)
    sched = _get_optimizer_param_scheduler(opt)
    args.iteration = 0
    if args.virtual_pipeline_model_parallel_size is not None:
        its = [build_train_valid_test_data_iterators(finetune.train_valid_test_datasets_provider)
               for _ in model]
        train_it = [i[0] for i in its]
    else:
        train_it = build_train_valid_test_data_iterators(
            finetune.train_valid_test_datasets_provider)[0]
    losses = []
    for _ in range(steps):
        ld, skipped, gnorm, _ = train_step(finetune.forward_step, train_it, model, opt, sched, args)
        v = gnorm.value() if hasattr(gnorm, "value") else gnorm  # LazyScalar
        gnorm = None if v is None else float(v)
        args.consumed_train_samples += args.global_batch_size
        if ld:
            losses.append((float(ld["lm loss"]), gnorm))
    return losses if state.is_pipeline_last_stage(ignore_virtual=True) else None


def _losses(res):
    out = [r for r in res if r]
    return out[0]


def _baseline(base, steps=3):
    return _losses(run_dist(_train, 1, base + ["--micro_batch_size", "2",
                                               "--global_batch_size", "4"], steps))


@pytest.fixture(scope="module")
def llama_ref():
    return _baseline(TINY_LLAMA)


@pytest.fixture(scope="module")
def gpt_ref():
    return _baseline(TINY_GPT)


def _check(ref, got, tol=2e-5):
    assert len(ref) == len(got)
    for (l0, g0), (l1, g1) in zip(ref, got):
        assert abs(l0 - l1) < tol * max(1.0, abs(l0)), (ref, got)
        assert abs(g0 - g1) < 1e-4 * max(1.0, abs(g0)), (ref, got)


def test_llama_loss_decreases(llama_ref):
    assert llama_ref[-1][0] < llama_ref[0][0]


@pytest.mark.parametrize("extra", [
    ["--tensor_model_parallel_size", "2"],
    ["--tensor_model_parallel_size", "2", "--sequence_parallel"],
    ["--tensor_model_parallel_size", "2", "--sequence_parallel", "--sp_regather_inputs"],
])
def test_llama_tensor_parallel(llama_ref, extra):
    got = _losses(run_dist(_train, 2, TINY_LLAMA + extra + ["--micro_batch_size", "2",
                                                             "--global_batch_size", "4"], 3))
    _check(llama_ref, got)


def test_llama_data_parallel(llama_ref):
    got = _losses(run_dist(_train, 2, TINY_LLAMA + ["--micro_batch_size", "1",
                                                     "--global_batch_size", "4"], 3))
    # dp=2 x mbs=1 x 2 microbatches consumes the same samples as dp=1 x mbs=1 x 4
    base = _losses(run_dist(_train, 1, TINY_LLAMA + ["--micro_batch_size", "1",
                                                      "--global_batch_size", "4"], 3))
    _check(base, got)


def test_llama_distributed_optimizer():
    argv = TINY_LLAMA + ["--micro_batch_size", "1", "--global_batch_size", "4"]
    base = _losses(run_dist(_train, 1, argv, 3))
    got = _losses(run_dist(_train, 2, argv + ["--use_distributed_optimizer"], 3))
    _check(base, got)


def test_gpt_tied_rotary_distributed_optimizer_param_gather():
    """Tied embeddings + rotary + no dropout + dist-opt at DP=2: the tied
    embedding sits in the held bucket, gathered and waited first, and the
    fused residual-norm path calls ``forward_residual`` directly, so the
    layer norms must wait for their own bucket's overlapped all-gather (with
    EMA_COMM_CHECK the gather is deferred: a missing wait reads stale shards)."""
    argv = TINY_GPT + ["--position_embedding_type", "rotary", "--micro_batch_size", "1",
                       "--global_batch_size", "4", "--ddp_bucket_size_mb", "0.02",
                       "--lr", "1e-2"]
    base = _losses(run_dist(_train, 1, argv, 3))
    got = _losses(run_dist(_train, 2, argv + ["--use_distributed_optimizer"], 3))
    # tight: a stale norm shard moved the step-2 grad norm by 4e-6 (relative)
    # and the loss by 5e-7 on this config; the waited path is exact to fp32 noise
    for (l0, g0), (l1, g1) in zip(base, got):
        assert abs(l0 - l1) < 2e-7 * abs(l0), (base, got)
        assert abs(g0 - g1) < 1e-6 * abs(g0), (base, got)


def test_llama_dp_concurrent_comm_groups():
    """DDP buckets issued round-robin on two communicators over the same DP
    ranks (--ddp_comm_groups 2, small buckets so there are many): all-reduce
    and reduce-scatter / all-gather (dist-opt) paths match DP=1."""
    argv = TINY_LLAMA + ["--micro_batch_size", "1", "--global_batch_size", "4",
                         "--ddp_bucket_size_mb", "0.05"]
    base = _losses(run_dist(_train, 1, argv, 3))
    for extra in ([], ["--use_distributed_optimizer"]):
        got = _losses(run_dist(_train, 2, argv + extra + ["--ddp_comm_groups", "2"], 3))
        _check(base, got)


def test_llama_pipeline_1f1b(llama_ref):
    got = _losses(run_dist(_train, 2, TINY_LLAMA + ["--pipeline_model_parallel_size", "2",
                                                     "--micro_batch_size", "2",
                                                     "--global_batch_size", "4"], 3))
    _check(llama_ref, got)


def test_llama_pipeline_interleaved():
    argv = TINY_LLAMA[:]
    argv[argv.index("--num_layers") + 1] = "4"
    base = _losses(run_dist(_train, 1, argv + ["--micro_batch_size", "1",
                                               "--global_batch_size", "4"], 3))
    got = _losses(run_dist(_train, 2, argv + ["--pipeline_model_parallel_size", "2",
                                              "--num_layers_per_virtual_pipeline_stage", "1",
                                              "--allow_interleaved_pp2",
                                              "--micro_batch_size", "1",
                                              "--global_batch_size", "4"], 3))
    _check(base, got)


def test_llama_tp_pp_dp():
    argv = TINY_LLAMA + ["--micro_batch_size", "1", "--global_batch_size", "4"]
    base = _losses(run_dist(_train, 1, argv, 2))
    got = _losses(run_dist(_train, 8, argv + ["--tensor_model_parallel_size", "2",
                                              "--pipeline_model_parallel_size", "2",
                                              "--sequence_parallel"], 2))
    _check(base, got, tol=5e-5)


@pytest.mark.parametrize("extra", [
    ["--tensor_model_parallel_size", "2"],
    ["--pipeline_model_parallel_size", "2"],
])
def test_gpt_parallel(gpt_ref, extra):
    got = _losses(run_dist(_train, 2, TINY_GPT + extra + ["--micro_batch_size", "2",
                                                           "--global_batch_size", "4"], 3))
    _check(gpt_ref, got)


# --------------------------------------------------------------------------
# Round-2 coverage: the BASELINE shapes in miniature, tied embeddings with
# DP > 1 (contribution counting), dist-opt with PP (embedding all-reduce
# before the reduce-scatter), SP with DP > 1 (no write into a bucket in
# flight: the race checker of parallel/comm.py is on for every test).

def _mb(m, g):
    return ["--micro_batch_size", str(m), "--global_batch_size", str(g)]


def _set(argv, flag, value):
    argv = list(argv)
    if flag in argv:
        argv[argv.index(flag) + 1] = value
    else:
        argv += [flag, value]
    return argv


@pytest.mark.parametrize("extra", [
    [],
    ["--use_distributed_optimizer"],
])
def test_gpt_tied_embeddings_data_parallel(extra):
    base = _losses(run_dist(_train, 1, TINY_GPT + _mb(1, 4), 3))
    got = _losses(run_dist(_train, 2, TINY_GPT + _mb(1, 4) + extra, 3))
    _check(base, got)


def test_gpt_pp_dp_distributed_optimizer():
    """Tied embeddings across PP stages + dist-opt: the embedding-group sum must
    precede the DP reduce-scatter."""
    base = _losses(run_dist(_train, 1, TINY_GPT + _mb(1, 4), 3))
    got = _losses(run_dist(_train, 4, TINY_GPT + _mb(1, 4) + [
        "--pipeline_model_parallel_size", "2", "--use_distributed_optimizer"], 3))
    _check(base, got)


def test_llama_sp_dp_distributed_optimizer():
    """SP norm-grad TP sums after the async DP reduce-scatter has completed."""
    base = _losses(run_dist(_train, 1, TINY_LLAMA + _mb(1, 4), 3))
    got = _losses(run_dist(_train, 4, TINY_LLAMA + _mb(1, 4) + [
        "--tensor_model_parallel_size", "2", "--sequence_parallel",
        "--use_distributed_optimizer"], 3))
    _check(base, got, tol=5e-5)


TINY_GQA = _set(_set(TINY_LLAMA, "--num_attention_heads", "8"), "--ffn_hidden_size", "128") + \
    ["--num_attention_heads_kv", "2"]


@pytest.mark.parametrize("tp", [2])
def test_llama_gqa_tensor_parallel_one_group_per_rank(tp):
    """70B-style GQA at TP = nkv: exactly one KV group per rank."""
    base = _losses(run_dist(_train, 1, TINY_GQA + _mb(2, 4), 3))
    got = _losses(run_dist(_train, tp, TINY_GQA + _mb(2, 4) + [
        "--tensor_model_parallel_size", str(tp), "--sequence_parallel"], 3))
    _check(base, got, tol=5e-5)


TINY_LLAMA8 = _set(TINY_LLAMA, "--num_attention_heads", "8")


@pytest.mark.parametrize("tp", [4, 8])
def test_llama_wide_tensor_parallel(tp):
    base = _losses(run_dist(_train, 1, TINY_LLAMA8 + _mb(2, 2), 2))
    got = _losses(run_dist(_train, tp, TINY_LLAMA8 + _mb(2, 2) + [
        "--tensor_model_parallel_size", str(tp), "--sequence_parallel"], 2))
    _check(base, got, tol=5e-5)


TINY_FALCON = ["--num_layers", "4", "--hidden_size", "64", "--num_attention_heads", "8",
               "--num_attention_heads_kv", "2", "--seq_length", "16",
               "--max_position_embeddings", "32", "--position_embedding_type", "rotary",
               "--parallel_attn", "--parallel_layernorm", "--hidden_dropout", "0.0",
               "--attention_dropout", "0.0", "--no_bias_gelu_fusion", "--no_bias_dropout_fusion",
               "--tokenizer_type", "NullTokenizer", "--synthetic_vocab_size", "250",
               "--make_vocab_size_divisible_by", "8", "--use_cpu_initialization",
               "--model_name", "falcon", "--lr", "1e-3", "--train_iters", "4", "--seed", "1234",
               "--log_interval", "1000", "--eval_iters", "0", "--eval_interval", "1000",
               "--synthetic_data", "--clip_grad", "1.0"]


def test_falcon_tp_pp_interleaved():
    """BASELINE config #4 in miniature: Falcon (parallel attn + parallel LN, GQA,
    tied embeddings) at TP=2 x PP=2 with the interleaved schedule."""
    base = _losses(run_dist(_train, 1, TINY_FALCON + _mb(1, 4), 3))
    got = _losses(run_dist(_train, 4, TINY_FALCON + _mb(1, 4) + [
        "--tensor_model_parallel_size", "2", "--pipeline_model_parallel_size", "2",
        "--num_layers_per_virtual_pipeline_stage", "1", "--allow_interleaved_pp2",
        "--sequence_parallel"], 3))
    _check(base, got, tol=5e-5)


def test_falcon_data_parallel_distributed_optimizer():
    base = _losses(run_dist(_train, 1, TINY_FALCON + _mb(1, 4), 3))
    got = _losses(run_dist(_train, 2, TINY_FALCON + _mb(1, 4) +
                           ["--use_distributed_optimizer"], 3))
    _check(base, got)


def test_llama_full_recompute_sp_distributed_activations():
    base = _losses(run_dist(_train, 1, TINY_LLAMA + _mb(2, 4), 3))
    got = _losses(run_dist(_train, 2, TINY_LLAMA + _mb(2, 4) + [
        "--tensor_model_parallel_size", "2", "--sequence_parallel",
        "--recompute_granularity", "full", "--recompute_method", "uniform",
        "--recompute_num_layers", "1", "--distribute_saved_activations"], 3))
    _check(base, got, tol=5e-5)


def test_llama_pp_distributed_optimizer():
    base = _losses(run_dist(_train, 1, TINY_LLAMA + _mb(1, 4), 3))
    got = _losses(run_dist(_train, 4, TINY_LLAMA + _mb(1, 4) + [
        "--pipeline_model_parallel_size", "2", "--use_distributed_optimizer"], 3))
    _check(base, got)


# --- context parallelism (--context_parallel_size): ring attention over
# consecutive DP ranks that hold the sequence chunks of the same samples ---
def test_llama_context_parallel(llama_ref):
    got = _losses(run_dist(_train, 2, TINY_LLAMA + ["--context_parallel_size", "2",
                                                     "--micro_batch_size", "2",
                                                     "--global_batch_size", "4"], 3))
    _check(llama_ref, got)


def test_gpt_context_parallel_absolute_positions(gpt_ref):
    """Learned absolute position embeddings read the chunk's GLOBAL positions."""
    got = _losses(run_dist(_train, 2, TINY_GPT + ["--context_parallel_size", "2",
                                                   "--micro_batch_size", "2",
                                                   "--global_batch_size", "4"], 3))
    _check(gpt_ref, got)


def test_llama_context_parallel_gqa_eod_mask():
    """GQA ring, and a loss mask that differs between the chunks (EOD tokens
    masked): the CP-summed token count keeps the loss the whole-sequence mean."""
    argv = TINY_LLAMA + ["--num_attention_heads_kv", "2", "--eod_mask_loss",
                         "--micro_batch_size", "1", "--global_batch_size", "2"]
    base = _losses(run_dist(_train, 1, argv, 3))
    got = _losses(run_dist(_train, 4, argv + ["--context_parallel_size", "4"], 3))
    _check(base, got)


def test_llama_cp_tp_dp_pp():
    """CP=2 composed with TP=2 + SP and DP=2 (8 ranks), and with PP=2 (4 ranks)."""
    argv = TINY_LLAMA + ["--micro_batch_size", "1", "--global_batch_size", "4"]
    base = _losses(run_dist(_train, 1, argv, 2))
    got = _losses(run_dist(_train, 8, argv + ["--tensor_model_parallel_size", "2",
                                              "--sequence_parallel",
                                              "--context_parallel_size", "2",
                                              "--use_distributed_optimizer"], 2))
    _check(base, got, tol=5e-5)
    got = _losses(run_dist(_train, 4, argv + ["--pipeline_model_parallel_size", "2",
                                              "--context_parallel_size", "2"], 2))
    _check(base, got, tol=5e-5)


def test_llama_context_parallel_document_masks():
    """--reset_attention_mask / --reset_position_ids (packed documents) under
    context parallelism: the ring masks earlier documents from the whole
    sequence's bounds; CP 2 and CP 4 train like CP 1.  A vocabulary of 8
    makes EOD (token 7) frequent, so documents cross the zig-zag pieces."""
    argv = [("8" if a == "250" else a) for a in TINY_LLAMA] + [
        "--reset_attention_mask", "--reset_position_ids",
        "--micro_batch_size", "2", "--global_batch_size", "4"]
    base = _losses(run_dist(_train, 1, argv, 3))
    for cp in (2, 4):
        got = _losses(run_dist(_train, cp, argv + ["--context_parallel_size", str(cp)], 3))
        _check(base, got)


@pytest.mark.parametrize("tp,pieces", [(2, "5,11"), (8, "1,3")])
def test_llama_sp_mlp_uneven_pieces(llama_ref, monkeypatch, tp, pieces):
    """The SP MLP pipeline with uneven pieces (layers._sp_mlp_pieces picks them
    where even pieces quantize the fc1 + GLU GEMM): forced here, it trains like
    TP = 1, with every collective's shapes checked (EMA_COMM_CHECK)."""
    monkeypatch.setenv("EMA_SP_MLP_PIECES", pieces)
    monkeypatch.setenv("EMA_COMM_CHECK", "1")
    argv = TINY_LLAMA if tp == 2 else TINY_LLAMA8
    base = llama_ref if tp == 2 else _losses(run_dist(_train, 1, TINY_LLAMA8 + _mb(2, 4), 3))
    mb = ["--micro_batch_size", "2", "--global_batch_size", "4"] if tp == 2 else _mb(2, 4)
    got = _losses(run_dist(_train, tp, argv + mb + ["--tensor_model_parallel_size", str(tp),
                                                    "--sequence_parallel"], 3))
    _check(base, got, tol=5e-5)


def _sp_gathers(rank, world, argv):
    import finetune
    init_framework(argv, finetune.extra_args)
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.parallel import comm
    from epfl_megatron_amd.training import (_setup_model_and_optimizer,
                                            build_train_valid_test_data_iterators, train_step)
    args = get_args()
    model, opt, sched = _setup_model_and_optimizer(finetune.model_provider,
                                                   ModelType.encoder_or_decoder, args=args)
    it = build_train_valid_test_data_iterators(finetune.train_valid_test_datasets_provider)[0]
    train_step(finetune.forward_step, it, model, opt, sched, args)
    comm.report(reset=True)
    train_step(finetune.forward_step, it, model, opt, sched, args)
    rep = comm.report()
    return {k: (v[0], v[1]) for k, v in rep.items() if k.endswith("/tp")}, args.num_layers


def test_sp_keeps_gathered_inputs_for_wgrad():
    """Kept SP gathers (default): the backward all-gathers no input of a
    column-parallel product (QKV, fc1, LM head) again: per micro-batch 2 full
    [s, b, h] all-gathers per layer + 1 for the LM head fewer;
    every other TP collective is unchanged."""
    argv = TINY_LLAMA + ["--tensor_model_parallel_size", "2", "--sequence_parallel",
                         "--micro_batch_size", "2", "--global_batch_size", "4"]
    kept, layers = run_dist(_sp_gathers, 2, argv)[0]
    regather, _ = run_dist(_sp_gathers, 2, argv + ["--sp_regather_inputs"])[0]
    n_micro, seq, mbs = 2, 16, 2
    hidden = int(TINY_LLAMA[TINY_LLAMA.index("--hidden_size") + 1])
    full = seq * mbs * hidden * 4  # one gathered [s, b, h] (fp32 params in the tiny run)
    extra = regather["all_gather/tp"][1] - kept["all_gather/tp"][1]
    assert extra == n_micro * (2 * layers + 1) * full, (kept, regather, full)
    for k in ("reduce_scatter/tp", "all_reduce/tp", "broadcast/tp"):
        assert regather[k] == kept[k]

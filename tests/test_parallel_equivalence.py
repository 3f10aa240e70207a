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

"""Checkpoint compatibility in both directions.

* A checkpoint written here loads in a process where ``epfl_megatron_amd`` is
  NOT importable and only the reference's ``megatron.model.enums`` exists (a
  5-enum stub with the reference's names and values): the args enums are
  pickled under the reference module path.
* Distributed-optimizer state is written in the reference's per-DP-rank layout
  (``shard_fp32_from_float16_groups`` + per-shard Adam state, cut by the
  reference buffer layout), so it reloads at another bucket size and another
  DP size and training continues exactly as if never interrupted.
* checkpoint_version < 2.0 fused-QKV row orders are migrated on load.
* Legacy pickled loss scalers (``fp16.loss_scaler.*``) deserialise under the
  weights-only loader.
"""
import io
import json
import os
import subprocess
import sys
import textwrap

import pytest
import torch

from dist_utils import run_dist, init_framework, TINY_LLAMA, TINY_GPT

REF_ENUMS_STUB = textwrap.dedent('''
    import enum

    class ModelType(enum.Enum):
        encoder_or_decoder = 1
        encoder_and_decoder = 2

    class LayerType(enum.Enum):
        encoder = 1
        decoder = 2

    class AttnType(enum.Enum):
        self_attn = 1
        cross_attn = 2

    class AttnMaskType(enum.Enum):
        padding = 1
        causal = 2

    class PositionEmbeddingType(enum.Enum):
        rotary = 1
        absolute = 2
''')

READER = textwrap.dedent('''
    import json, sys, torch
    try:
        import epfl_megatron_amd  # must NOT be importable here
        print(json.dumps({"error": "framework importable"})); sys.exit(0)
    except ImportError:
        pass
    sd = torch.load(sys.argv[1], map_location="cpu", weights_only=False)
    a = sd["args"]
    out = {"pe_module": type(a.position_embedding_type).__module__,
           "pe": a.position_embedding_type.name,
           "model_type": str(getattr(a, "model_type", None)),
           "num_layers": a.num_layers, "version": sd["checkpoint_version"],
           "iteration": sd["iteration"]}
    flat = {}
    def walk(prefix, d):
        for k, v in d.items():
            if isinstance(v, dict):
                walk(prefix + k + ".", v)
            elif torch.is_tensor(v):
                flat[prefix + k] = float(v.double().sum())
    walk("", sd["model"])
    out["tensors"] = flat
    print(json.dumps(out))
''')


def _flat_sums(d, prefix=""):
    out = {}
    for k, v in d.items():
        if isinstance(v, dict):
            out.update(_flat_sums(v, prefix + k + "."))
        elif torch.is_tensor(v):
            out[prefix + k] = float(v.double().sum())
    return out


def _train_and_save(rank, world, argv, ckdir, iters):
    import finetune
    init_framework(argv + ["--save", ckdir, "--save_interval", str(iters),
                           "--train_iters", str(iters)], finetune.extra_args)
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.training import pretrain
    args = get_args()
    pretrain(args, finetune.train_valid_test_datasets_provider, finetune.model_provider,
             ModelType.encoder_or_decoder, finetune.forward_step)
    return True


def test_reference_loader_reads_our_checkpoint(tmp_path):
    ck = str(tmp_path / "ck")
    run_dist(_train_and_save, 1, TINY_LLAMA + ["--micro_batch_size", "1",
                                               "--global_batch_size", "2"], ck, 1)
    path = os.path.join(ck, "iter_0000001", "mp_rank_00", "model_optim_rng.pt")
    raw = open(path, "rb").read()
    assert b"epfl_megatron_amd" not in raw  # nothing of ours is referenced by the pickle
    stub = tmp_path / "stub"
    (stub / "megatron" / "model").mkdir(parents=True)
    (stub / "megatron" / "__init__.py").write_text("")
    (stub / "megatron" / "model" / "__init__.py").write_text("")
    (stub / "megatron" / "model" / "enums.py").write_text(REF_ENUMS_STUB)
    (stub / "reader.py").write_text(READER)
    env = dict(os.environ, PYTHONPATH=str(stub))
    out = subprocess.run([sys.executable, str(stub / "reader.py"), path], cwd=str(stub), env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = json.loads(out.stdout.strip().splitlines()[-1])
    assert "error" not in got, got
    assert got["pe_module"] == "megatron.model.enums" and got["pe"] == "rotary"
    assert got["num_layers"] == 2 and got["version"] == 3.0 and got["iteration"] == 1
    # the same tensors our own (weights-only) loader reads
    from epfl_megatron_amd.checkpointing import safe_load
    ours = _flat_sums(safe_load(path)["model"])
    assert got["tensors"].keys() == ours.keys()
    for k in ours:
        assert got["tensors"][k] == pytest.approx(ours[k], rel=1e-12, abs=1e-12), k


# ------------------------------------------------- distributed-optimizer state
def _train_losses(rank, world, argv, steps, load=None, save=None):
    import finetune
    extra = []
    if load:
        extra += ["--load", load]
    if save:
        extra += ["--save", save, "--save_interval", str(steps)]
    init_framework(argv + extra, finetune.extra_args)
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.checkpointing import save_checkpoint
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.parallel import state
    from epfl_megatron_amd.training import (_setup_model_and_optimizer,
                                            build_train_valid_test_data_iterators, train_step)
    args = get_args()
    model, opt, sched = _setup_model_and_optimizer(finetune.model_provider,
                                                   ModelType.encoder_or_decoder, args=args)
    it = build_train_valid_test_data_iterators(finetune.train_valid_test_datasets_provider)[0]
    losses = []
    for _ in range(steps):
        ld, _, gn, _ = train_step(finetune.forward_step, it, model, opt, sched, args)
        args.consumed_train_samples += args.global_batch_size
        args.iteration += 1
        losses.append((float(ld["lm loss"]), float(gn)))
    if save:
        save_checkpoint(args.iteration, model, opt, sched)
    return losses if state.get_data_parallel_rank() == 0 else None


BASE = TINY_LLAMA + ["--micro_batch_size", "1", "--global_batch_size", "4", "--train_iters", "8",
                     "--use_distributed_optimizer"]


@pytest.fixture(scope="module")
def distopt_ckpt(tmp_path_factory):
    """2 steps at DP=2 with tiny (many) buckets, saved; plus the 4-step straight run."""
    d = str(tmp_path_factory.mktemp("distopt"))
    small = BASE + ["--ddp_bucket_size_mb", "0.002"]
    run_dist(_train_losses, 2, small, 2, None, d)
    straight = [r for r in run_dist(_train_losses, 2, small, 4) if r][0]
    return d, straight


def test_distopt_checkpoint_layout_is_reference(distopt_ckpt):
    d, _ = distopt_ckpt
    from epfl_megatron_amd.checkpointing import safe_load
    sds = [safe_load(os.path.join(d, "iter_0000002", f"mp_rank_00_{r:03d}", "optim.pt"))
           for r in range(2)]
    for r, sd in enumerate(sds):
        o = sd["optimizer"]
        assert set(o) >= {"optimizer", "shard_fp32_from_float16_groups"}
        n_groups = len(o["optimizer"]["param_groups"])
        assert len(o["shard_fp32_from_float16_groups"]) == n_groups
        assert o["layout"]["dp_size"] == 2 and o["layout"]["dp_rank"] == r
    # the two ranks' shards partition every parameter exactly once (fp32 CPU model:
    # no fp32-from-fp16 copies, as in the reference; count the Adam state shards)
    tot = sum(st["exp_avg"].numel() for sd in sds
              for st in sd["optimizer"]["optimizer"]["state"].values())
    assert tot == sds[0]["optimizer"]["layout"]["chunk_numel"][0]


@pytest.mark.parametrize("world,extra", [
    (2, []),                                  # default (512 MiB) buckets: different layout
    (1, []),                                  # DP 2 -> 1
    (4, ["--ddp_bucket_size_mb", "0.01"]),    # DP 2 -> 4, other small buckets
])
def test_distopt_checkpoint_reshards(distopt_ckpt, world, extra):
    d, straight = distopt_ckpt
    resumed = [r for r in run_dist(_train_losses, world, BASE + extra, 2, d) if r][0]
    for (l0, g0), (l1, g1) in zip(straight[2:], resumed):
        assert abs(l0 - l1) < 2e-5 * max(1.0, abs(l0)), (straight, resumed)
        assert abs(g0 - g1) < 1e-4 * max(1.0, abs(g0)), (straight, resumed)


# ------------------------------------------------------ old QKV row orders
def _qkv_migration(rank, world, version):
    import finetune
    init_framework(TINY_GPT + ["--micro_batch_size", "1"], finetune.extra_args)
    from epfl_megatron_amd.checkpointing import fix_query_key_value_ordering
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.training import get_model
    model = get_model(finetune.model_provider, ModelType.encoder_or_decoder,
                      wrap_with_ddp=False)[0]
    attn = model.language_model.encoder.layers[0].self_attention
    nh, hd = attn.num_attention_heads_per_partition, attn.hidden_size_per_attention_head
    ref = {n: p.detach().clone() for n, p in model.named_parameters() if "query_key_value" in n}
    with torch.no_grad():  # write the pre-2.0 layout of the same weights
        for n, p in model.named_parameters():
            if "query_key_value" in n:
                rest = p.shape[1:]
                t = p.view(nh, 3, hd, *rest)
                t = t.transpose(0, 1) if version == 0 else t.permute(0, 2, 1, *range(3, 3 + len(rest)))
                p.copy_(t.contiguous().view(p.shape))
                assert p.dim() == 1 or not torch.equal(p, ref[n])
    fix_query_key_value_ordering(model, version)
    return all(torch.equal(p, ref[n]) for n, p in model.named_parameters() if n in ref)


@pytest.mark.parametrize("version", [0, 1.0])
def test_qkv_ordering_migration(version):
    assert run_dist(_qkv_migration, 1, version)[0]


# -------------------------------------------------- legacy loss-scaler shim
def test_legacy_loss_scaler_checkpoint_loads(tmp_path):
    from epfl_megatron_amd.checkpointing import safe_load
    from epfl_megatron_amd.fp16_deprecated import loss_scaler as ls
    import types
    legacy = types.ModuleType("fp16.loss_scaler")
    pkg = types.ModuleType("fp16")
    old_mod = ls.DynamicLossScaler.__module__
    sys.modules["fp16"], sys.modules["fp16.loss_scaler"] = pkg, legacy
    legacy.DynamicLossScaler = ls.DynamicLossScaler
    ls.DynamicLossScaler.__module__ = "fp16.loss_scaler"
    try:
        buf = io.BytesIO()
        torch.save({"optimizer": {"loss_scaler": ls.DynamicLossScaler(init_scale=2 ** 12)},
                    "w": torch.arange(3.0)}, buf)
        path = tmp_path / "old.pt"
        path.write_bytes(buf.getvalue())
    finally:
        ls.DynamicLossScaler.__module__ = old_mod
        del sys.modules["fp16"], sys.modules["fp16.loss_scaler"]
    sd = safe_load(str(path))
    assert sd["optimizer"]["loss_scaler"].cur_scale == 2 ** 12
    assert torch.equal(sd["w"], torch.arange(3.0))

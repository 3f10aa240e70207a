"""Reference oracle for the distributed-optimizer shard layout.

``oracle_plan`` re-derives, independently of ``optim/optimizer.py``, which
slice of which parameter each DP rank's ``optim.pt`` holds and in which order,
the way the reference builds it:

* the grad buffer of a model chunk is packed from its END in
  ``module.parameters()`` order (``megatron/model/distributed.py:121-157``:
  a per-dtype countdown of element counts),
* it is cut into ``ceil(numel / dp)``-element world ranges, one per DP rank
  (``megatron/optimizer/distrib_optimizer.py:119-164``),
* each parameter overlapping a rank's range contributes the sub-range
  ``(gbuf_world, gbuf_local, param)`` (``distrib_optimizer.py:63-116``),
* the shards are listed per optimizer group (weight-decay group first, then
  biases / 1-D params; empty groups squeezed), chunk by chunk, in parameter
  order (``distrib_optimizer.py:190-224``, ``megatron/optimizer/__init__.py:13-60``).

The tests check the framework's plan against the oracle at DP 1/2/4/8 for the
tiny GPT and Llama models, check the CONTENT of the shards written at DP 2 and
4 against the DP 1 state cut by the oracle's ranges, and check that a shard
whose sizes do not match the layout refuses to load.
"""
import math
import os

import pytest
import torch

from dist_utils import run_dist, init_framework, TINY_LLAMA, TINY_GPT


def oracle_plan(chunks, dp, r):
    """``chunks``: per model chunk, ``[(name, numel, ndim)]`` of the parameters
    that require grad, in ``module.parameters()`` order.  Returns the squeezed
    groups, each ``[(chunk, name, param_lo, param_hi)]``."""
    wd, no_wd = set(), set()
    for ci, params in enumerate(chunks):
        for name, _, ndim in params:
            (no_wd if name.endswith(".bias") or ndim == 1 else wd).add((ci, name))
    order = [g for g in (wd, no_wd) if g]
    groups = [[] for _ in order]
    for ci, params in enumerate(chunks):
        total = sum(n for _, n, _ in params)
        # countdown packing: the first parameter sits at the buffer's end
        left, index = total, {}
        for name, n, _ in params:
            left -= n
            index[name] = (left, left + n)
        size = int(math.ceil(total / dp))
        w_lo, w_hi = r * size, min(total, r * size + size)
        for name, _, _ in params:
            p_lo, p_hi = index[name]
            loc_lo, loc_hi = max(0, p_lo - w_lo), min(w_hi - w_lo, p_hi - w_lo)
            if loc_hi > loc_lo:
                sub = max(0, w_lo - p_lo)
                gi = next(i for i, g in enumerate(order) if (ci, name) in g)
                groups[gi].append((ci, name, sub, sub + loc_hi - loc_lo))
    return [g for g in groups if g]


# ---------------------------------------------------------------- oracle self-test
def test_oracle_partitions_every_parameter_exactly_once():
    chunks = [[("a.weight", 10, 2), ("a.bias", 3, 1), ("b.weight", 7, 2)],
              [("c.weight", 5, 2), ("c.bias", 2, 1)]]
    for dp in (1, 2, 3, 4, 8):
        seen = {}
        for r in range(dp):
            for g in oracle_plan(chunks, dp, r):
                for ci, name, lo, hi in g:
                    seen.setdefault((ci, name), []).append((lo, hi))
        for ci, params in enumerate(chunks):
            for name, n, _ in params:
                rs = sorted(seen[(ci, name)])
                assert rs[0][0] == 0 and rs[-1][1] == n
                assert all(a[1] == b[0] for a, b in zip(rs, rs[1:])), (dp, name, rs)
    # hand-checked: chunk 0 = 20 elements packed [b.weight 0-7][a.bias 7-10][a.weight 10-20];
    # DP 2 rank 0 owns buffer 0-10 -> b.weight whole and a.bias whole
    assert oracle_plan(chunks[:1], 2, 0) == [[(0, "b.weight", 0, 7)], [(0, "a.bias", 0, 3)]]
    assert oracle_plan(chunks[:1], 2, 1) == [[(0, "a.weight", 0, 10)]]
    # DP 3: ranges of 7 -> rank 1 owns 7-14: a.bias whole and a.weight[0:4]
    assert oracle_plan(chunks[:1], 3, 1) == [[(0, "a.weight", 0, 4)], [(0, "a.bias", 0, 3)]]


# ------------------------------------------------ framework plan == oracle plan
def _plans(rank, world, argv, dps):
    import finetune
    init_framework(argv, finetune.extra_args)
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.training import _setup_model_and_optimizer
    args = get_args()
    model, opt, _ = _setup_model_and_optimizer(finetune.model_provider,
                                               ModelType.encoder_or_decoder, args=args)
    chunks, names = [], {}
    for ci, c in enumerate(opt.chunks):
        params = []
        for name, p in c.ddp.module.named_parameters():
            if p.requires_grad:
                params.append((name, p.numel(), p.dim()))
                names[p] = name
        chunks.append(params)
    out = {}
    for dp in dps:
        for r in range(dp):
            ours = [[(ci, names[p], lo, hi) for ci, p, lo, hi in entries]
                    for _, entries in opt._ref_plan(dp, r)]
            out[(dp, r)] = ours
    return chunks, out


@pytest.mark.parametrize("name,argv", [
    ("llama", TINY_LLAMA),
    ("gpt", TINY_GPT),
])
def test_framework_plan_matches_reference_oracle(name, argv):
    chunks, plans = run_dist(_plans, 1, argv + ["--micro_batch_size", "1",
                                                "--use_distributed_optimizer"],
                             (1, 2, 4, 8))[0]
    for (dp, r), ours in plans.items():
        assert ours == oracle_plan(chunks, dp, r), (name, dp, r)


# -------------------------------------------- shard CONTENT at DP 2 / 4 vs DP 1
def _train_save(rank, world, argv, ckdir, steps):
    import finetune
    init_framework(argv + ["--save", ckdir, "--save_interval", "1000"], finetune.extra_args)
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.checkpointing import save_checkpoint
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.training import (_setup_model_and_optimizer,
                                            build_train_valid_test_data_iterators, train_step)
    args = get_args()
    model, opt, sched = _setup_model_and_optimizer(finetune.model_provider,
                                                   ModelType.encoder_or_decoder, args=args)
    it = build_train_valid_test_data_iterators(finetune.train_valid_test_datasets_provider)[0]
    for _ in range(steps):
        train_step(finetune.forward_step, it, model, opt, sched, args)
        args.consumed_train_samples += args.global_batch_size
        args.iteration += 1
    save_checkpoint(args.iteration, model, opt, sched)
    return [[(n, p.numel(), p.dim()) for n, p in c.ddp.module.named_parameters()
             if p.requires_grad] for c in opt.chunks]


DIST = TINY_LLAMA + ["--micro_batch_size", "1", "--global_batch_size", "8",
                     "--use_distributed_optimizer", "--ddp_bucket_size_mb", "0.01"]


def _shards(d, dp):
    from epfl_megatron_amd.checkpointing import safe_load
    return [safe_load(os.path.join(d, "iter_0000002", f"mp_rank_00_{r:03d}",
                                   "optim.pt"))["optimizer"] for r in range(dp)]


@pytest.fixture(scope="module")
def dp1_state(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("dp1"))
    chunks = run_dist(_train_save, 1, DIST, d, 2)[0]
    sd = _shards(d, 1)[0]
    (plan,) = [oracle_plan(chunks, 1, 0)]
    full, idx = {}, 0
    for g in plan:
        for ci, name, lo, hi in g:
            assert (lo, hi) == (0, dict((n, k) for n, k, _ in chunks[ci])[name])
            full[(ci, name)] = sd["optimizer"]["state"][idx]
            idx += 1
    return chunks, full


@pytest.mark.parametrize("dp", [2, 4])
def test_shard_contents_follow_reference_ranges(dp1_state, tmp_path, dp):
    chunks, full = dp1_state
    d = str(tmp_path / f"dp{dp}")
    assert run_dist(_train_save, dp, DIST, d, 2)[0] == chunks
    for r, sd in enumerate(_shards(d, dp)):
        plan = oracle_plan(chunks, dp, r)
        groups = sd["optimizer"]["param_groups"]
        assert len(groups) == len(plan)
        idx = 0
        for g, want in zip(groups, plan):
            assert list(g["params"]) == list(range(idx, idx + len(want)))
            for ci, name, lo, hi in want:
                st = sd["optimizer"]["state"][idx]
                for key in ("exp_avg", "exp_avg_sq"):
                    ref = full[(ci, name)][key].reshape(-1)[lo:hi]
                    got = st[key].reshape(-1)
                    assert got.numel() == hi - lo, (r, name, key)
                    # same math at another DP size: only the gradient summation
                    # order differs; a shifted slice would be off by O(1)
                    torch.testing.assert_close(got, ref, rtol=2e-4, atol=1e-9 + 1e-4 * ref.abs().max().item())
                idx += 1
        assert idx == len(sd["optimizer"]["state"])


# ------------------------------------------------------ a mismatched file refuses
def _load_expect_refusal(rank, world, argv, ckdir):
    import finetune
    init_framework(argv + ["--load", ckdir], finetune.extra_args)
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.training import _setup_model_and_optimizer
    try:
        _setup_model_and_optimizer(finetune.model_provider, ModelType.encoder_or_decoder,
                                   args=get_args())
    except SystemExit as e:  # load_checkpoint: "Unable to load optimizer ... exiting"
        return f"exit {e.code}"
    except RuntimeError as e:
        return str(e)
    return None


def test_mismatched_shard_refuses_to_load(tmp_path):
    d = str(tmp_path / "ck")
    run_dist(_train_save, 2, DIST, d, 2)
    path = os.path.join(d, "iter_0000002", "mp_rank_00_001", "optim.pt")
    sd = torch.load(path, map_location="cpu", weights_only=True)
    st = sd["optimizer"]["optimizer"]["state"]
    k = sorted(st)[0]
    st[k]["exp_avg"] = st[k]["exp_avg"].reshape(-1)[1:].clone()  # one element short
    torch.save(sd, path)
    out = run_dist(_load_expect_refusal, 2, DIST, d)
    # every rank reads every DP peer's shard: both refuse, naming the bad shard
    assert all(o and "shard 1" in o and "expected" in o for o in out), out

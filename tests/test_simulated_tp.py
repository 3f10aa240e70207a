"""--simulated_tensor_parallel_size: one TP rank of a TP=N model in one process
(the 1-GPU proxies of the TP configurations)."""
import torch

from dist_utils import run_dist, init_framework, TINY_LLAMA


def _sim_rank(rank, world, n):
    import finetune
    init_framework(TINY_LLAMA + ["--micro_batch_size", "2", "--num_attention_heads", "8",
                                 "--simulated_tensor_parallel_size", str(n),
                                 "--sequence_parallel"], finetune.extra_args)
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.parallel import comm, state
    from epfl_megatron_amd.training import (_setup_model_and_optimizer,
                                            build_train_valid_test_data_iterators, train_step)
    args = get_args()
    out = {"tp": state.get_tensor_model_parallel_world_size(), "sp": args.sequence_parallel}
    g = state.get_tensor_model_parallel_group()
    x = torch.arange(6, dtype=torch.float32).view(3, 2)
    full = torch.empty(3 * n, 2)
    comm.all_gather_into(full, x, group=g)
    # emulation: every simulated rank's slot holds this rank's shard (finite
    # stand-ins written on every call, as a real all-gather writes its whole
    # output), no reduction kernel
    out["ag"] = all(torch.equal(full[3 * i:3 * i + 3], x) for i in range(n))
    # a persistent scratch buffer: peers' slots written on the first gather
    # into that range only, afterwards just the own slot
    from epfl_megatron_amd.parallel.buffers import get_global_memory_buffer
    sc = get_global_memory_buffer().get_tensor((3 * n, 2), torch.float32, "loopback-test")
    comm.all_gather_into(sc, x, group=g)
    first = all(torch.equal(sc[3 * i:3 * i + 3], x) for i in range(n))
    comm.all_gather_into(sc, x + 100, group=g)
    out["ag_scratch"] = first and torch.equal(sc[:3], x + 100) and all(
        torch.equal(sc[3 * i:3 * i + 3], x) for i in range(1, n))
    # another user takes the same buffer with another view and writes it (here
    # NaN): the next hand-out in the first view is a new generation, so the
    # peers' slots are refilled instead of trusted
    other = get_global_memory_buffer().get_tensor((n, 6), torch.float32, "loopback-test")
    other.fill_(float("nan"))
    sc = get_global_memory_buffer().get_tensor((3 * n, 2), torch.float32, "loopback-test")
    comm.all_gather_into(sc, x, group=g)
    out["ag_regen"] = bool(torch.isfinite(sc).all()) and all(
        torch.equal(sc[3 * i:3 * i + 3], x) for i in range(n))
    # SP gathers kept for the backward come from a pool under the loopback: a
    # buffer is handed out again only once nothing references it, and its
    # peers' slots are written once per buffer
    pool = get_global_memory_buffer()
    k1 = pool.get_kept((3 * n, 2), torch.float32, "cpu")
    k2 = pool.get_kept((3 * n, 2), torch.float32, "cpu")
    busy = k1.data_ptr() != k2.data_ptr()
    comm.all_gather_into(k1, x, group=g)
    p1 = k1.data_ptr()
    saved = k1[:3]  # a view (as autograd's saved tensor) keeps the buffer taken
    del k1
    k3 = pool.get_kept((3 * n, 2), torch.float32, "cpu")
    busy = busy and k3.data_ptr() not in (p1, k2.data_ptr())
    del saved, k3
    k4 = pool.get_kept((3 * n, 2), torch.float32, "cpu")
    comm.all_gather_into(k4, x + 100, group=g)
    out["kept_pool"] = busy and k4.data_ptr() == p1 and torch.equal(k4[:3], x + 100) and all(
        torch.equal(k4[3 * i:3 * i + 3], x) for i in range(1, n))
    del k2, k4
    parts = torch.arange(n * 6, dtype=torch.float32).view(n * 3, 2)
    rs = torch.empty(3, 2)
    comm.reduce_scatter_into(rs, parts, group=g)
    out["rs"] = torch.equal(rs, parts[:3])
    model, opt, sched = _setup_model_and_optimizer(finetune.model_provider,
                                                   ModelType.encoder_or_decoder, args=args)
    shapes = {k: tuple(p.shape) for k, p in model[0].named_parameters()}
    out["qkv"] = next(v for k, v in shapes.items() if "query_key_value" in k)
    out["fc1"] = next(v for k, v in shapes.items() if "dense_h_to_4h" in k)
    it = build_train_valid_test_data_iterators(finetune.train_valid_test_datasets_provider)[0]
    comm.report(reset=True)
    ld, _, _, _ = train_step(finetune.forward_step, it, model, opt, sched, args)
    out["loss"] = float(ld["lm loss"])
    out["comm"] = {k: v[0] for k, v in comm.report().items() if k.endswith("/tp")}
    return out


def test_simulated_tp_rank_shapes_and_loopback():
    out = run_dist(_sim_rank, 1, 4)[0]
    assert out["tp"] == 4 and out["sp"]
    assert out["ag"] and out["rs"] and out["ag_scratch"] and out["ag_regen"] and out["kept_pool"]
    # h 64, 8 heads of 8 -> 2 heads per rank: qkv 3 * 2 * 8 = 48 rows; ffn 128 -> 2 * 32
    assert out["qkv"] == (48, 64) and out["fc1"] == (64, 64)
    assert out["loss"] == out["loss"] and out["loss"] > 0
    # SP: two all-gathers (qkv, fc1) and two reduce-scatters (dense, fc2) per layer
    # and micro-batch in the forward at least
    assert out["comm"].get("all_gather/tp", 0) >= 4 and out["comm"].get("reduce_scatter/tp", 0) >= 4

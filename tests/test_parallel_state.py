"""Rank -> group topology (reference tests/test_parallel_state.py, on gloo/CPU)."""
import torch
import torch.distributed as dist

from dist_utils import run_dist


def _topology(rank, world, tp, pp, vpp):
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from epfl_megatron_amd.parallel import state
    state.initialize_model_parallel(tp, pp, vpp)
    dp = world // (tp * pp)
    out = dict(
        tp_rank=state.get_tensor_model_parallel_rank(),
        tp_world=state.get_tensor_model_parallel_world_size(),
        pp_rank=state.get_pipeline_model_parallel_rank(),
        pp_world=state.get_pipeline_model_parallel_world_size(),
        dp_rank=state.get_data_parallel_rank(),
        dp_world=state.get_data_parallel_world_size(),
        tp_src=state.get_tensor_model_parallel_src_rank(),
        first=state.is_pipeline_first_stage(ignore_virtual=True),
        last=state.is_pipeline_last_stage(ignore_virtual=True),
        next=state.get_pipeline_model_parallel_next_rank(),
        prev=state.get_pipeline_model_parallel_prev_rank(),
        emb=state.is_rank_in_embedding_group(ignore_virtual=True),
    )
    # collectives within each group actually work
    t = torch.ones(1)
    dist.all_reduce(t, group=state.get_tensor_model_parallel_group())
    out["tp_sum"] = t.item()
    t = torch.ones(1)
    dist.all_reduce(t, group=state.get_data_parallel_group())
    out["dp_sum"] = t.item()
    t = torch.ones(1)
    dist.all_reduce(t, group=state.get_model_parallel_group())
    out["mp_sum"] = t.item()
    state.destroy_model_parallel()
    return out


def test_topology_tp2_pp2_dp2():
    world, tp, pp = 8, 2, 2
    res = run_dist(_topology, world, tp, pp, None)
    for rank, r in enumerate(res):
        # global_rank = pp_rank*(tp*dp) + dp_rank*tp + tp_rank
        dp = world // (tp * pp)
        assert rank == r["pp_rank"] * (tp * dp) + r["dp_rank"] * tp + r["tp_rank"]
        assert r["tp_world"] == tp and r["pp_world"] == pp and r["dp_world"] == dp
        assert r["tp_src"] == (rank // tp) * tp
        assert r["first"] == (r["pp_rank"] == 0) and r["last"] == (r["pp_rank"] == pp - 1)
        assert r["next"] == (rank + world // pp) % world
        assert r["prev"] == (rank - world // pp) % world
        assert r["emb"]  # with pp=2 every stage is first or last
        assert r["tp_sum"] == tp and r["dp_sum"] == dp and r["mp_sum"] == tp * pp


def test_topology_tp4_pp1():
    res = run_dist(_topology, 4, 4, 1, None)
    assert [r["tp_rank"] for r in res] == [0, 1, 2, 3]
    assert all(r["dp_world"] == 1 for r in res)


def test_rank_grid_layout():
    from epfl_megatron_amd.parallel.state import rank_grid
    g = rank_grid(16, 2, 4)
    assert g.shape == (4, 2, 2)
    assert g[1, 1, 0] == 1 * 4 + 1 * 2 + 0


def _cp_topology(rank, world):
    from epfl_megatron_amd.parallel import state
    dist.init_process_group("gloo", rank=rank, world_size=world)
    state.initialize_model_parallel(2, 1, context_parallel_size=2)
    return (dist.get_process_group_ranks(state.get_context_parallel_group()),
            state.get_context_parallel_rank(), state.get_data_sample_parallel_rank(),
            state.get_data_sample_parallel_world_size(), state.get_data_parallel_world_size())


def test_context_parallel_groups_tp2_cp2_dp2():
    """grid [pp=1, dp=4, tp=2]: CP pairs consecutive DP indices, so rank r
    shares its sequence with r +- tp; DP sample index = dp index // 2."""
    res = run_dist(_cp_topology, 8)
    for rank, (ranks, cpr, sr, ssize, dsize) in enumerate(res):
        dp_idx, tp_idx = rank // 2, rank % 2
        c0 = dp_idx // 2 * 2
        assert ranks == [c0 * 2 + tp_idx, (c0 + 1) * 2 + tp_idx]
        assert cpr == dp_idx % 2 and sr == dp_idx // 2
        assert ssize == 2 and dsize == 4

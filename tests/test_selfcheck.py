"""Startup collective self-check (parallel/selfcheck.py) on gloo: it passes on
every group of a TP x PP x DP grid with concurrent DP communicators, and it
fails loudly when a collective does not behave as the framework assumes."""
from dist_utils import run_dist, init_framework, TINY_LLAMA


def _init_and_count(rank, world, argv):
    import finetune
    init_framework(argv, finetune.extra_args)
    from epfl_megatron_amd.parallel.selfcheck import collective_selfcheck
    return collective_selfcheck(verbose=False)


def test_selfcheck_passes_on_3d_grid():
    argv = TINY_LLAMA + ["--tensor_model_parallel_size", "2", "--pipeline_model_parallel_size",
                         "2", "--ddp_comm_groups", "2", "--micro_batch_size", "1",
                         "--global_batch_size", "4"]
    counts = run_dist(_init_and_count, 8, argv)
    # env agreement 1 + 2 DP communicators x 6 + TP 6 + PP 1 on every rank
    assert counts == [20] * 8


def test_selfcheck_passes_with_context_parallel():
    argv = TINY_LLAMA + ["--tensor_model_parallel_size", "2", "--context_parallel_size", "2",
                         "--micro_batch_size", "1", "--global_batch_size", "4"]
    counts = run_dist(_init_and_count, 4, argv)
    # env agreement 1 + DP (2 ranks) 6 + TP 6 + CP 6 (no pipeline)
    assert counts == [19] * 4


def _broken_avg(rank, world, argv):
    import finetune
    init_framework(argv + ["--no_comm_selfcheck"], finetune.extra_args)
    from epfl_megatron_amd.parallel import comm, selfcheck
    real = comm.reduce_scatter_into

    def summing(output, inp, group=None, async_op=False, op="sum"):  # ignores AVG
        return real(output, inp, group=group, async_op=async_op, op="sum")

    comm.reduce_scatter_into = summing
    try:
        selfcheck.collective_selfcheck(verbose=False)
    except RuntimeError as e:
        return "reduce_scatter(AVG" in str(e)
    finally:
        comm.reduce_scatter_into = real
    return False


def test_selfcheck_detects_wrong_semantics():
    argv = TINY_LLAMA + ["--micro_batch_size", "1", "--global_batch_size", "4"]
    assert run_dist(_broken_avg, 2, argv) == [True, True]


def _mismatched_knob(rank, world, argv):
    import os
    import finetune
    # rank 1 would split its SP all-gathers in 4 pieces, rank 0 in 2: RCCL
    # would hang mid-step, so the startup check must refuse
    os.environ["EMA_SP_CHUNKS"] = str(2 + 2 * rank)
    os.environ["EMA_TRACE"] = str(rank)  # rank-local: allowed to differ
    try:
        init_framework(argv, finetune.extra_args)
    except RuntimeError as e:
        msg = str(e)
        return "EMA_SP_CHUNKS=['2', '4']" in msg and "EMA_TRACE" not in msg
    return False


def test_selfcheck_refuses_mismatched_env_knobs():
    argv = TINY_LLAMA + ["--tensor_model_parallel_size", "2", "--micro_batch_size", "1",
                         "--global_batch_size", "4"]
    assert run_dist(_mismatched_knob, 2, argv) == [True, True]


def test_structural_env_filters_local_knobs():
    from epfl_megatron_amd.parallel.selfcheck import structural_env
    env = {"EMA_SP_CHUNKS": "4", "EMA_FUSED_MLP": "0", "EMA_TRACE": "1", "EMA_GEMM_GM": "8",
           "EMA_WGRAD_GN": "4", "EMA_NEW_KNOB": "x", "PATH": "/bin"}
    assert structural_env(env) == {"EMA_FUSED_MLP": "0", "EMA_NEW_KNOB": "x",
                                   "EMA_SP_CHUNKS": "4"}

"""Forward + backward of the bench.py training step, for in-step hardware
counters (rocprofv3 --pmc).

The model, shapes, data and parallel config are bench.py's (same argument
parser: ``--seq_len``, ``--micro_batch``, ``--proxy`` ...); the step runs
``--warmup`` + ``--steps`` forward/backward passes over all micro-batches
WITHOUT the optimizer step.  Reason: under
``rocprofv3 --pmc`` the host process segfaulted inside the profiler at the
first grad-norm kernel launch (profiles/r6e_pmc_gemms.txt:68,
gpurun_out r7g_pmc1.log), after the forward/backward kernels had been
counted; the optimizer's kernels are not the subject of the counter tables
(wgrad / NT GEMMs / FlashAttention / hipBLASLt).  The counted kernels run in
the step's own memory state and order, which is what "in-step" means here.

    rocprofv3 --pmc ... --kernel-include-regex 'wgrad_k|gemm_nt6_k|fa_|Cijk' \\
        -- python3 scripts/pmc_step.py --steps 1 --warmup 1
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main():
    a = bench._parse(sys.argv[1:])
    import torch
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(bench._free_port()))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    if not torch.cuda.is_available():
        raise SystemExit("pmc_step.py needs a GPU")
    cfg, shape = bench._resolve(a, 1)
    fargv, _ = bench._framework_argv(a, cfg, shape, 1, True)

    import finetune
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.initialize import initialize_megatron
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.parallel.pipeline.schedules import get_forward_backward_func
    from epfl_megatron_amd.training import (_setup_model_and_optimizer,
                                            build_train_valid_test_data_iterators)

    initialize_megatron(finetune.extra_args, {"tokenizer_type": "NullTokenizer"}, args_list=fargv)
    args = get_args()
    chunks, optimizer, sched = _setup_model_and_optimizer(finetune.model_provider,
                                                         ModelType.encoder_or_decoder, args=args)
    train_it = build_train_valid_test_data_iterators(finetune.train_valid_test_datasets_provider,
                                                     args)[0]
    for m in chunks:
        m.train()
    from epfl_megatron_amd.global_vars import get_timers as _timers
    fwd_bwd = get_forward_backward_func()

    def passes(n):
        for _ in range(n):
            for m in chunks:
                if hasattr(m, "zero_grad_buffer"):
                    m.zero_grad_buffer()
            fwd_bwd(finetune.forward_step, train_it, chunks, optimizer, _timers(),
                    forward_only=False)
        torch.cuda.synchronize()

    passes(a.warmup)  # (warm-up without the optimizer too: see above)
    passes(a.steps)
    print(f"pmc_step: {a.steps} forward/backward pass(es) done", flush=True)


if __name__ == "__main__":
    main()

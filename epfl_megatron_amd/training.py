"""Training driver: ``pretrain`` / ``train_step`` / ``evaluate``
(reference ``megatron/training.py``; provider-function API unchanged).

MI355X additions: the log line also reports tokens/s (per GPU and total),
model TFLOP/s per GPU and MFU against ``--peak_tflops`` (dense bf16 peak);
``get_model`` wraps every chunk in the bucketed, backward-overlapped DDP.
"""
import math
import sys
import time
from datetime import datetime

import torch
import torch.distributed as dist

from . import global_vars
from .global_vars import (get_args, get_current_global_batch_size, get_num_microbatches,
                          get_signal_handler, get_tensorboard_writer, get_timers,
                          update_num_microbatches)
from .checkpointing import load_checkpoint, save_checkpoint
from .models.enums import ModelType
from .models.module import Float16Module
from .optim import get_megatron_optimizer, OptimizerParamScheduler
from .optim.optimizer import LazyScalar
from .parallel import comm
from .utils.trace import set_tracing, trace_range
from .parallel import state
from .parallel.ddp import DistributedDataParallel as LocalDDP
from .parallel.pipeline.schedules import get_forward_backward_func
from .parallel.tensor import set_defaults_if_not_set_tensor_model_parallel_attributes
from .parallel.tensor.layers import fallback_report, new_weight_transpose_generation
from .utils.misc import (calc_params_l2_norm, check_adlr_autoresume_termination, print_all_nodes,
                         print_rank_0, print_rank_last, report_memory, unwrap_model)
from .utils.flops import flops_per_token
from .data.samplers import build_pretraining_data_loader

_TRAIN_START_TIME = time.time()


def print_datetime(string):
    if dist.is_initialized():
        dist.barrier()
    print_rank_0(f"[{string}] datetime: {datetime.now().strftime('%Y-%m-%d %H:%M:%S')} ")


def _device():
    return torch.cuda.current_device() if torch.cuda.is_available() else "cpu"


def pretrain(args, train_valid_test_dataset_provider, model_provider_func, model_type,
             forward_step_func, process_non_loss_data_func=None):
    global _TRAIN_START_TIME
    t = torch.tensor([_TRAIN_START_TIME], dtype=torch.float64,
                     device=_device() if args.distributed_backend != "gloo" else "cpu")
    comm.all_reduce(t, op=dist.ReduceOp.MIN)
    _TRAIN_START_TIME = t.item()
    print_rank_0(f"time to initialize megatron (seconds): {time.time() - _TRAIN_START_TIME:.3f}")
    print_datetime("after megatron is initialized")
    timers = get_timers()
    timers("model-and-optimizer-setup", log_level=0).start(barrier=True)
    model, optimizer, opt_param_scheduler = _setup_model_and_optimizer(
        model_provider_func, model_type, args=args)
    timers("model-and-optimizer-setup").stop()
    print_datetime("after model, optimizer, and learning rate scheduler are built")
    timers("train/valid/test-data-iterators-setup", log_level=0).start(barrier=True)
    if args.virtual_pipeline_model_parallel_size is not None:
        its = [build_train_valid_test_data_iterators(train_valid_test_dataset_provider, args)
               for _ in range(len(model))]
        train_it = [i[0] for i in its]
        valid_it = [i[1] for i in its]
        test_it = [i[2] for i in its]
    else:
        train_it, valid_it, test_it = build_train_valid_test_data_iterators(
            train_valid_test_dataset_provider, args)
    timers("train/valid/test-data-iterators-setup").stop()
    print_datetime("after dataloaders are built")
    print_rank_0("done with setup ...")
    timers.log(["model-and-optimizer-setup", "train/valid/test-data-iterators-setup"],
               barrier=True)
    print_rank_0("training ...")
    iteration = 0
    if args.do_train and args.train_iters > 0:
        iteration = _train(args, forward_step_func, model, optimizer, opt_param_scheduler,
                           train_it, valid_it, process_non_loss_data_func)
    print_datetime("after training is done")
    if args.do_valid:
        evaluate_and_print_results("the end of training for val data", forward_step_func,
                                   valid_it, model, iteration, process_non_loss_data_func,
                                   verbose=False, args=args)
    if args.save and iteration != 0:
        save_checkpoint(iteration, model, optimizer, opt_param_scheduler)
    if args.do_test:
        evaluate_and_print_results("the end of training for test data", forward_step_func,
                                   test_it, model, 0, process_non_loss_data_func, verbose=True,
                                   args=args)
    return model, optimizer, opt_param_scheduler


def _update_train_iters(args):
    if args.rampup_batch_size is None:
        args.train_iters = args.train_samples // args.global_batch_size
        return
    iterations, consumed = 0, 0
    while consumed <= int(args.rampup_batch_size[2]):
        update_num_microbatches(consumed, consistency_check=False)
        consumed += get_current_global_batch_size()
        iterations += 1
    update_num_microbatches(0, consistency_check=False)
    iterations += (args.train_samples - consumed) // args.global_batch_size
    args.train_iters = iterations
    print_rank_0(f"setting training iterations to {args.train_iters}")


def get_model(model_provider_func, model_type=ModelType.encoder_or_decoder, wrap_with_ddp=True,
              args=None):
    args = args or get_args()
    args.model_type = model_type
    pp = state.get_pipeline_model_parallel_world_size()
    if pp > 1 and args.virtual_pipeline_model_parallel_size is not None:
        if model_type == ModelType.encoder_and_decoder:
            raise AssertionError("Interleaved schedule not supported for encoder-decoder models")
        model = []
        for i in range(args.virtual_pipeline_model_parallel_size):
            state.set_virtual_pipeline_model_parallel_rank(i)
            m = model_provider_func(pre_process=state.is_pipeline_first_stage(),
                                    post_process=state.is_pipeline_last_stage())
            m.model_type = model_type
            model.append(m)
        state.set_virtual_pipeline_model_parallel_rank(0)
    else:
        pre, post = state.is_pipeline_first_stage(), state.is_pipeline_last_stage()
        add_enc, add_dec = True, False
        if model_type == ModelType.encoder_and_decoder and pp > 1:
            if args.pipeline_model_parallel_split_rank is None:
                raise AssertionError("Split rank needs to be specified for encoder-decoder")
            rank = state.get_pipeline_model_parallel_rank()
            split = args.pipeline_model_parallel_split_rank
            pre = rank == 0 or rank == split
            post = rank == split - 1 or rank == pp - 1
            add_enc = state.is_pipeline_stage_before_split()
            add_dec = state.is_pipeline_stage_after_split()
            m = model_provider_func(pre_process=pre, post_process=post, add_encoder=add_enc,
                                    add_decoder=add_dec)
        else:
            m = model_provider_func(pre_process=pre, post_process=post)
        m.model_type = model_type
        model = [m]
    for m in model:
        for p in m.parameters():
            set_defaults_if_not_set_tensor_model_parallel_attributes(p)
    if state.get_data_parallel_rank() == 0:
        n = sum(sum(p.nelement() for p in m.parameters()) for m in model)
        print(f" > number of parameters on (tensor, pipeline) model parallel rank "
              f"({state.get_tensor_model_parallel_rank()}, "
              f"{state.get_pipeline_model_parallel_rank()}): {n}", flush=True)
    if torch.cuda.is_available():
        model = [m.cuda(torch.cuda.current_device()) for m in model]
    if args.fp16 or args.bf16:
        model = [Float16Module(m, args) for m in model]
    if wrap_with_ddp:
        if args.DDP_impl == "torch":
            from torch.nn.parallel import DistributedDataParallel as TorchDDP
            dev = torch.cuda.current_device() if torch.cuda.is_available() else None
            model = [TorchDDP(m, device_ids=[dev] if dev is not None else None,
                              output_device=dev, process_group=state.get_data_parallel_group())
                     for m in model]
        elif args.DDP_impl == "local":
            model = [LocalDDP(m, args.accumulate_allreduce_grads_in_fp32,
                              args.use_contiguous_buffers_in_local_ddp,
                              bucket_size_mb=args.ddp_bucket_size_mb,
                              overlap_grad_reduce=args.overlap_grad_reduce,
                              use_distributed_optimizer=args.use_distributed_optimizer,
                              overlap_param_gather=args.overlap_param_gather)
                     for m in model]
            if args.data_parallel_random_init:
                for m in model:
                    m.broadcast_params()
        else:
            raise NotImplementedError(f"Unknown DDP implementation specified: {args.DDP_impl}.")
    return model


def _get_optimizer_param_scheduler(optimizer, args=None):
    args = args or get_args()
    if args.train_iters:
        if args.lr_decay_iters is None:
            args.lr_decay_iters = args.train_iters
        decay = args.lr_decay_iters * args.global_batch_size
        wd_incr = args.train_iters * args.global_batch_size
        warm = args.lr_warmup_fraction * decay if args.lr_warmup_fraction is not None \
            else args.lr_warmup_iters * args.global_batch_size
    elif args.train_samples:
        _update_train_iters(args)
        if args.lr_decay_samples is None:
            args.lr_decay_samples = args.train_samples
        decay = args.lr_decay_samples
        wd_incr = args.train_samples
        warm = args.lr_warmup_fraction * decay if args.lr_warmup_fraction is not None \
            else args.lr_warmup_samples
    else:
        raise Exception("either train_iters or train_samples should be provided.")
    return OptimizerParamScheduler(
        optimizer, max_lr=args.lr, min_lr=args.min_lr, lr_warmup_steps=warm,
        lr_decay_steps=decay, lr_decay_style=args.lr_decay_style,
        start_wd=args.start_weight_decay, end_wd=args.end_weight_decay, wd_incr_steps=wd_incr,
        wd_incr_style=args.weight_decay_incr_style,
        use_checkpoint_opt_param_scheduler=args.use_checkpoint_opt_param_scheduler,
        override_opt_param_scheduler=args.override_opt_param_scheduler)


def _setup_model_and_optimizer(model_provider_func, model_type, no_wd_decay_cond=None,
                               scale_lr_cond=None, lr_mult=1.0, args=None):
    args = args or get_args()
    model = get_model(model_provider_func, model_type, args=args)
    optimizer = get_megatron_optimizer(model, no_wd_decay_cond, scale_lr_cond, lr_mult)
    opt_param_scheduler = _get_optimizer_param_scheduler(optimizer, args)
    if args.load is not None:
        timers = get_timers()
        timers("load-checkpoint", log_level=0).start(barrier=True)
        args.iteration = load_checkpoint(model, optimizer, opt_param_scheduler)
        timers("load-checkpoint").stop(barrier=True)
        timers.log(["load-checkpoint"])
    else:
        args.iteration = 0
    if args.iteration == 0 and len(unwrap_model(model)) == 1 and \
            hasattr(unwrap_model(model)[0], "init_state_dict_from_bert"):
        unwrap_model(model)[0].init_state_dict_from_bert()
    return model, optimizer, opt_param_scheduler


def train_step(forward_step_func, data_iterator, model, optimizer, opt_param_scheduler, args):
    timers = get_timers()
    new_weight_transpose_generation()
    if args.DDP_impl == "local":
        for m in model:
            m.zero_grad_buffer()
    optimizer.zero_grad()
    fwd_bwd = get_forward_backward_func()
    timers("forward-backward", log_level=1).start(barrier=args.barrier_with_L1_time)
    losses_reduced = fwd_bwd(forward_step_func, data_iterator, model, optimizer, timers,
                             forward_only=False)
    timers("forward-backward").stop()
    if args.empty_unused_memory_level >= 1 and torch.cuda.is_available():
        torch.cuda.empty_cache()
    with trace_range("reduce-grads"):
        optimizer.reduce_model_grads(args, timers)
    timers("optimizer", log_level=1).start(barrier=args.barrier_with_L1_time)
    with trace_range("optimizer-step"):
        update_successful, grad_norm, num_zeros = optimizer.step(args, timers)
    timers("optimizer").stop()
    # The skip decision is made on the device; the scheduler advances now and
    # is rolled back by the optimizer if the step turns out to be skipped.
    increment = get_num_microbatches() * args.micro_batch_size * args.data_parallel_size
    opt_param_scheduler.step(increment=increment)
    optimizer.register_scheduler_step(opt_param_scheduler, increment)
    skipped_iter = LazyScalar(lambda: 0 if update_successful else 1)
    if args.empty_unused_memory_level >= 2 and torch.cuda.is_available():
        torch.cuda.empty_cache()
    if state.is_pipeline_last_stage(ignore_virtual=True):
        loss_reduced = {}
        for key in losses_reduced[0]:
            vals = [x[key] for x in losses_reduced]
            loss_reduced[key] = sum(vals) / len(vals)
        return loss_reduced, skipped_iter, grad_norm, num_zeros
    return {}, skipped_iter, grad_norm, num_zeros


def training_log(loss_dict, total_loss_dict, learning_rate, iteration, loss_scale,
                 skipped_iter, grad_norm, params_norm, num_zeros_in_grad, report_memory_flag,
                 consumed_samples=None, num_microbatches=None):
    """Log one iteration.  The loop logs an iteration one step late (so reading
    its lazy device scalars never stalls the queue); ``consumed_samples`` and
    ``num_microbatches`` are the values captured when it was enqueued (None:
    read the live globals, for direct callers)."""
    args = get_args()
    if consumed_samples is None:
        consumed_samples = args.consumed_train_samples
    if num_microbatches is None:
        num_microbatches = get_num_microbatches()
    timers = get_timers()
    writer = get_tensorboard_writer()
    # lazy device->host values of the step being logged (one iteration old)
    skipped_iter = int(skipped_iter)
    grad_norm = grad_norm.value() if isinstance(grad_norm, LazyScalar) else grad_norm
    if callable(loss_scale):
        loss_scale = loss_scale()
    adv, skp, nan = "advanced iterations", "skipped iterations", "nan iterations"
    if not skipped_iter:
        total_loss_dict[adv] = total_loss_dict.get(adv, 0) + 1
    elif adv not in total_loss_dict:
        total_loss_dict[adv] = 0
    total_loss_dict[skp] = total_loss_dict.get(skp, 0) + skipped_iter
    got_nan = False
    for key, val in loss_dict.items():
        if not skipped_iter:
            total_loss_dict[key] = total_loss_dict.get(key, torch.zeros(1, device=val.device
                                                                        if torch.is_tensor(val)
                                                                        else "cpu")) + val
        else:
            v = float(val)
            got_nan = got_nan or v in (float("inf"), -float("inf")) or v != v
    total_loss_dict[nan] = total_loss_dict.get(nan, 0) + int(got_nan)

    timers_to_log = ["forward-backward", "forward-compute", "backward-compute", "batch-generator",
                     "forward-recv", "forward-send", "backward-recv", "backward-send",
                     "forward-send-forward-recv", "forward-send-backward-recv",
                     "backward-send-forward-recv", "backward-send-backward-recv",
                     "forward-backward-send-forward-backward-recv", "layernorm-grads-all-reduce",
                     "embedding-grads-all-reduce", "grads-all-reduce", "grads-reduce-scatter",
                     "params-all-gather", "optimizer-copy-to-main-grad",
                     "optimizer-unscale-and-check-inf", "optimizer-clip-main-grad",
                     "optimizer-count-zeros", "optimizer-inner-step",
                     "optimizer-copy-main-to-model-params", "optimizer"]
    normalizer = iteration % args.log_interval or args.log_interval
    batch_size = args.micro_batch_size * args.data_parallel_size * num_microbatches
    total_iterations = total_loss_dict[adv] + total_loss_dict[skp]

    if writer and (iteration % args.tensorboard_log_interval == 0):
        if args.log_learning_rate_to_tensorboard:
            writer.add_scalar("learning-rate", learning_rate, iteration)
            writer.add_scalar("learning-rate vs samples", learning_rate, consumed_samples)
        if args.log_batch_size_to_tensorboard:
            writer.add_scalar("batch-size", batch_size, iteration)
        for key, val in loss_dict.items():
            writer.add_scalar(key, float(val), iteration)
            writer.add_scalar(key + " vs samples", float(val), consumed_samples)
        if args.log_loss_scale_to_tensorboard:
            writer.add_scalar("loss-scale", loss_scale, iteration)
        if args.log_world_size_to_tensorboard:
            writer.add_scalar("world-size", args.world_size, iteration)
        if grad_norm is not None:
            writer.add_scalar("grad-norm", grad_norm, iteration)
        if num_zeros_in_grad is not None:
            writer.add_scalar("num-zeros", num_zeros_in_grad, iteration)
        if params_norm is not None:
            writer.add_scalar("params-norm", params_norm, iteration)
        if args.log_memory_to_tensorboard and torch.cuda.is_available():
            writer.add_scalar("mem-reserved-bytes", torch.cuda.memory_reserved(), iteration)
            writer.add_scalar("mem-allocated-bytes", torch.cuda.memory_allocated(), iteration)
        if args.log_timers_to_tensorboard:
            timers.write(timers_to_log, writer, iteration, normalizer=total_iterations)

    if iteration % args.log_interval == 0:
        elapsed = timers("interval-time").elapsed(barrier=True)
        per_iter = elapsed / max(total_iterations, 1)
        tokens = batch_size * args.seq_length
        tok_s = tokens / per_iter if per_iter > 0 else 0.0
        tok_s_gpu = tok_s / args.world_size
        tflops_gpu = tok_s_gpu * flops_per_token(args) / 1e12
        mfu = tflops_gpu / args.peak_tflops
        if writer and args.log_timers_to_tensorboard:
            writer.add_scalar("iteration-time", per_iter, iteration)
        s = f" iteration {iteration:8d}/{args.train_iters:8d} |"
        s += f" consumed samples: {consumed_samples:12d} |"
        s += f" elapsed time per iteration (ms): {per_iter * 1000.0:.1f} |"
        s += f" learning rate: {learning_rate:.3E} |"
        s += f" global batch size: {batch_size:5d} |"
        for key in list(total_loss_dict.keys()):
            if key in (adv, skp, nan):
                continue
            avg = float(total_loss_dict[key]) / float(max(1, total_loss_dict[adv]))
            if avg > 0.0:
                s += f" {key}: {avg:.6E} |"
            total_loss_dict[key] = torch.zeros(1, device=_device())
        s += f" loss scale: {loss_scale:.1f} |"
        if grad_norm is not None:
            s += f" grad norm: {grad_norm:.3f} |"
        if num_zeros_in_grad is not None:
            s += f" num zeros: {num_zeros_in_grad:.1f} |"
        if params_norm is not None:
            s += f" params norm: {params_norm:.3f} |"
        s += f" number of skipped iterations: {total_loss_dict[skp]:3d} |"
        s += f" number of nan iterations: {total_loss_dict[nan]:3d} |"
        if args.log_throughput:
            s += (f" tokens/s/GPU: {tok_s_gpu:.1f} | tokens/s: {tok_s:.1f} |"
                  f" TFLOP/s/GPU: {tflops_gpu:.1f} | MFU: {100.0 * mfu:.2f}% |")
        total_loss_dict[adv] = 0
        total_loss_dict[skp] = 0
        total_loss_dict[nan] = 0
        print_all_nodes(s)
        if writer and args.log_throughput:
            writer.add_scalar("throughput/tokens-per-sec-per-gpu", tok_s_gpu, iteration)
            writer.add_scalar("throughput/mfu", mfu, iteration)
        if report_memory_flag and learning_rate > 0.0:
            report_memory(f"(after {iteration} iterations)")
            report_memory_flag = False
        timers.log(timers_to_log, normalizer=args.log_interval)
        # correctness checks that run whatever the timing level: a one-shot
        # xGMI collective that timed out produced NaN output (raise now), and
        # GPU GEMMs that fell back to torch math are reported
        comm.check_xgmi()
        fb = fallback_report()
        if fb:
            print_rank_last(" GEMM kernel fallbacks (cumulative): " + ", ".join(
                f"{k}: {v}" for k, v in fb.items()))
        if args.timing_log_level >= 1:
            rep = comm.report()
            if rep:
                print_rank_last(" collectives (per interval): " + comm.format_report(rep))
    return report_memory_flag


def save_checkpoint_and_time(iteration, model, optimizer, opt_param_scheduler):
    timers = get_timers()
    timers("save-checkpoint", log_level=0).start(barrier=True)
    save_checkpoint(iteration, model, optimizer, opt_param_scheduler)
    timers("save-checkpoint").stop(barrier=True)
    timers.log(["save-checkpoint"])


def _train(args, forward_step_func, model, optimizer, opt_param_scheduler, train_data_iterator,
           valid_data_iterator, process_non_loss_data_func):
    timers = get_timers()
    from .initialize import write_args_to_tensorboard
    write_args_to_tensorboard()
    for m in model:
        m.train()
    total_loss_dict = {}
    iteration = args.iteration
    comm.set_timing(args.timing_log_level >= 2)
    if args.timing_log_level >= 2:  # roctx / torch.profiler ranges (utils/trace.py)
        set_tracing(True)
    timers("interval-time", log_level=0).start(barrier=True)
    print_datetime("before the start of training step")
    report_memory_flag = True
    pending_log = []

    def flush_log():
        nonlocal report_memory_flag
        while pending_log:
            entry, kw = pending_log.pop(0)
            report_memory_flag = training_log(*entry, report_memory_flag=report_memory_flag, **kw)

    while iteration < args.train_iters:
        update_num_microbatches(args.consumed_train_samples)
        step_microbatches = get_num_microbatches()
        args.curr_iteration = iteration
        loss_dict, skipped_iter, grad_norm, num_zeros = train_step(
            forward_step_func, train_data_iterator, model, optimizer, opt_param_scheduler, args)
        iteration += 1
        args.consumed_train_samples += args.data_parallel_size * \
            args.micro_batch_size * step_microbatches
        # Log the PREVIOUS iteration now that this one is enqueued: reading its
        # loss / grad norm / skip flag then never stalls the GPU queue.
        flush_log()
        if optimizer.grad_scaler:
            scale_t = optimizer.get_loss_scale().detach().clone()
            loss_scale = (lambda t=scale_t: float(t.item()))
        else:
            loss_scale = 1.0
        params_norm = None
        if args.log_params_norm:
            optimizer.wait_param_sync()
            params_norm = calc_params_l2_norm(model)
        pending_log.append(((loss_dict, total_loss_dict, optimizer.param_groups[0]["lr"],
                             iteration, loss_scale, skipped_iter, grad_norm, params_norm,
                             num_zeros),
                            {"consumed_samples": args.consumed_train_samples,
                             "num_microbatches": step_microbatches}))
        if args.adlr_autoresume and iteration % args.adlr_autoresume_interval == 0:
            flush_log()
            check_adlr_autoresume_termination(iteration, model, optimizer, opt_param_scheduler)
        if args.eval_interval and iteration % args.eval_interval == 0 and args.do_valid:
            flush_log()
            evaluate_and_print_results(f"iteration {iteration}", forward_step_func,
                                       valid_data_iterator, model, iteration,
                                       process_non_loss_data_func, verbose=False, args=args)
        writer = get_tensorboard_writer()
        if hasattr(writer, "flush_all"):
            writer.flush_all()
        saved = False
        if args.exit_signal_handler:
            if any(get_signal_handler().signals_received()):
                flush_log()
                save_checkpoint_and_time(iteration, model, optimizer, opt_param_scheduler)
                print_datetime("exiting program after receiving SIGTERM.")
                sys.exit()
        if args.save and args.save_interval and iteration % args.save_interval == 0:
            flush_log()
            save_checkpoint_and_time(iteration, model, optimizer, opt_param_scheduler)
            saved = True
        if args.exit_duration_in_mins:
            train_time = (time.time() - _TRAIN_START_TIME) / 60.0
            done = torch.tensor([int(train_time > args.exit_duration_in_mins)],
                                device=_device() if args.distributed_backend != "gloo" else "cpu")
            comm.all_reduce(done, op="max")
            if done.item():
                flush_log()
                if not saved:
                    save_checkpoint_and_time(iteration, model, optimizer, opt_param_scheduler)
                print_datetime(f"exiting program after {train_time} minutes")
                sys.exit()
        if args.exit_interval and iteration % args.exit_interval == 0:
            flush_log()
            if not saved:
                save_checkpoint_and_time(iteration, model, optimizer, opt_param_scheduler)
            dist.barrier()
            print_datetime(f"exiting program at iteration {iteration}")
            sys.exit()
    flush_log()
    optimizer.resolve_pending()
    optimizer.wait_param_sync()
    return iteration


def evaluate(forward_step_func, data_iterator, model, process_non_loss_data_func, verbose=False):
    args = get_args()
    for m in model:
        m.eval()
    total = {}
    with torch.no_grad():
        it = 0
        while it < args.eval_iters:
            it += 1
            if verbose and args.rank == 0:
                print_rank_0(f"Evaluating iter {it}/{args.eval_iters}")
            fwd_bwd = get_forward_backward_func()
            losses = fwd_bwd(forward_step_func, data_iterator, model, optimizer=None, timers=None,
                             forward_only=True)
            if args.empty_unused_memory_level >= 1 and torch.cuda.is_available():
                torch.cuda.empty_cache()
            if state.is_pipeline_last_stage(ignore_virtual=True):
                for ld in losses:
                    for k, v in ld.items():
                        total[k] = total.get(k, 0.0) + v
            args.consumed_valid_samples += args.data_parallel_size * \
                args.micro_batch_size * get_num_microbatches()
        collected = None
        if process_non_loss_data_func is not None and state.is_pipeline_last_stage():
            collected = fwd_bwd(forward_step_func, data_iterator, model, optimizer=None,
                                timers=None, forward_only=True, collect_non_loss_data=True)
    for m in model:
        m.train()
    for k in total:
        total[k] /= args.eval_iters * get_num_microbatches()
    return total, collected


def evaluate_and_print_results(prefix, forward_step_func, data_iterator, model, iteration,
                               process_non_loss_data_func, verbose=False, args=None):
    writer = get_tensorboard_writer()
    total, collected = evaluate(forward_step_func, data_iterator, model,
                                process_non_loss_data_func, verbose)
    s = f" validation loss at {prefix} | "
    for k, v in total.items():
        v = float(v)
        ppl = math.exp(min(20, v))
        s += f"{k} value: {v:.6E} | {k} PPL: {ppl:.6E} | "
        if writer:
            writer.add_scalar(f"{k} validation", v, iteration)
            writer.add_scalar(f"{k} validation vs samples", v, args.consumed_train_samples)
            if args.log_validation_ppl_to_tensorboard:
                writer.add_scalar(f"{k} validation ppl", ppl, iteration)
    if process_non_loss_data_func is not None and writer and collected is not None:
        process_non_loss_data_func(collected, iteration, writer)
    length = len(s) + 1
    print_rank_last("-" * length)
    print_rank_last(s)
    print_rank_last("-" * length)
    return total


def cyclic_iter(it):
    while True:
        for x in it:
            yield x


def build_train_valid_test_data_iterators(build_train_valid_test_datasets_provider, args=None):
    """Datasets are built on TP-rank 0 only; the do_train/valid/test flags are
    broadcast over the TP group (reference training.py:855-939)."""
    args = args or get_args()
    train_dl = valid_dl = test_dl = None
    print_rank_0("> building train, validation, and test datasets ...")
    if args.iteration > 0 and args.consumed_train_samples == 0:
        if args.train_samples is not None:
            raise AssertionError("only backward compatiblity support for iteration-based training")
        args.consumed_train_samples = args.iteration * args.global_batch_size
    if args.iteration > 0 and args.consumed_valid_samples == 0 and args.train_samples is None:
        args.consumed_valid_samples = (args.iteration // args.eval_interval) * \
            args.eval_iters * args.global_batch_size
    dev = _device() if args.distributed_backend != "gloo" else "cpu"
    if state.get_tensor_model_parallel_rank() == 0:
        train_samples = args.train_samples if args.train_samples else \
            args.train_iters * args.global_batch_size
        eval_iters = (args.train_iters // args.eval_interval + 1) * args.eval_iters \
            if args.eval_interval else 0
        sizes = [train_samples, eval_iters * args.global_batch_size,
                 args.eval_iters * args.global_batch_size]
        print_rank_0(" > datasets target sizes (minimum size):")
        print_rank_0(f"    train:      {sizes[0]}")
        print_rank_0(f"    validation: {sizes[1]}")
        print_rank_0(f"    test:       {sizes[2]}")
        train_ds, valid_ds, test_ds = build_train_valid_test_datasets_provider(sizes)
        train_dl = build_pretraining_data_loader(train_ds, args.consumed_train_samples)
        valid_dl = build_pretraining_data_loader(valid_ds, args.consumed_valid_samples)
        test_dl = build_pretraining_data_loader(test_ds, 0)
        flags = torch.tensor([int(train_dl is not None and args.train_iters > 0),
                              int(valid_dl is not None and args.eval_iters > 0),
                              int(test_dl is not None and args.eval_iters > 0)],
                             dtype=torch.long, device=dev)
    else:
        flags = torch.zeros(3, dtype=torch.long, device=dev)
    if state.get_tensor_model_parallel_world_size() > 1:
        comm.broadcast(flags, state.get_tensor_model_parallel_src_rank(),
                       group=state.get_tensor_model_parallel_group())
    args.do_train, args.do_valid, args.do_test = (bool(x) for x in flags.tolist())
    dl_type = args.dataloader_type

    def _it(dl):
        if dl is None:
            return None
        return iter(dl) if dl_type == "single" else iter(cyclic_iter(dl))

    return _it(train_dl), _it(valid_dl), _it(test_dl)

"""Headline benchmark: Llama-2-7B bf16 training throughput on N MI355X (one node).

Metric (BASELINE.json): tokens/s (+ MFU) for Llama-2-7B bf16; the default
preset is pure data parallelism with the distributed optimizer (weak scaling:
each GPU processes a fixed per-GPU batch).  The model is the real Llama-2-7B
architecture (32 layers, h=4096, 32 heads, ffn 11008, vocab 32000, RMSNorm,
SwiGLU, RoPE, untied head) with random init; data is synthetic tokens (a
learnable walk along a fixed random permutation of the vocabulary, so the
reported loss falls; no corpus / network).  Every timed step is a complete
training step through the framework: forward, backward, bucketed RCCL gradient
reduce-scatter overlapped with the backward, grad-norm clipping, fused AdamW
update, parameter all-gather (overlapped with the next forward).

``value`` is the whole-job aggregate tokens/s; ``vs_baseline`` compares the
per-GPU rate with the reference's published A100 figure (BASELINE.md P1':
~890 tokens/s/GPU for Llama-2-7B, seq 1024).

Launch (driver contract):
    python bench.py --gpus N --steps K --warmup W      # spawns N ranks itself
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

When started without torchrun and ``--gpus N > 1`` the parent spawns N child
processes (one per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their env)
BEFORE anything touches the GPU, waits for them and exits with their status.

Other BASELINE configs, one command each (need >= tp*pp GPUs):
    --preset llama7b-tp8-seq4096     Llama-2-7B, TP=8 (SP), seq 4096
    --preset falcon40b-tp4-pp2       Falcon-40B, TP=4 x PP=2 interleaved, 8 micro-batches
    --preset llama70b-tp8            Llama-2-70B, TP=8 (SP), full recompute, dist-opt
    --preset llama70b-tp8-budget     the same with the memory-model recompute policy (260 GB)
    --preset llama7b-cp8-seq32k      Llama-2-7B, seq 32768 split over 8 GPUs (context parallel;
                                     ring verified on gloo and on one GPU, not yet over RCCL)
1-GPU per-rank proxies of the TP configs (TP rank 0 of the real model built by
--simulated_tensor_parallel_size: per-rank GEMM / attention shapes, s/tp-row
norms and residuals under SP, TP collectives looped back locally and reported
with an analytic xGMI time; NOT the BASELINE metric, labelled "proxy"):
    --proxy llama7b-tp8 | llama70b-tp8 | falcon40b-tp4-pp2
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REF_TOKENS_PER_SEC_PER_GPU = 890.0  # BASELINE.md P1' (8x A100, seq 1024)
BASELINE_METRIC = "tokens/sec/GPU + MFU, Llama-2 7B bf16 TP/PP/DP at 1/2/4/8 MI355X"  # BASELINE.json

MODELS = {
    "llama2-7b": dict(family="llama2", L=32, h=4096, nh=32, nkv=None, ffn=11008, vocab=32000),
    "llama2-13b": dict(family="llama2", L=40, h=5120, nh=40, nkv=None, ffn=13824, vocab=32000),
    "llama2-70b": dict(family="llama2", L=80, h=8192, nh=64, nkv=8, ffn=28672, vocab=32000),
    "falcon-7b": dict(family="falcon", L=32, h=4544, nh=71, nkv=1, ffn=None, vocab=65024,
                      parallel_layernorm=False),
    "falcon-40b": dict(family="falcon", L=60, h=8192, nh=128, nkv=8, ffn=None, vocab=65024,
                       parallel_layernorm=True),
    "tiny": dict(family="llama2", L=2, h=256, nh=4, nkv=None, ffn=688, vocab=32000),
}

PRESETS = {
    # BASELINE config #2 (the headline): Llama-2-7B, pure DP (+ dist-opt at N > 1).
    # 16 x 8 = 128 sequences per GPU per step: a global batch of 1024 at 8 GPUs,
    # the reference's own P1 setting (gbs 1000 of seq 1024).
    "llama7b-dp": dict(model="llama2-7b", tp=1, pp=1, seq=1024, mbs=16, nmicro=8),
    # config #3
    "llama7b-tp8-seq4096": dict(model="llama2-7b", tp=8, pp=1, seq=4096, mbs=4, nmicro=4,
                                sp=True),
    # config #4
    "falcon40b-tp4-pp2": dict(model="falcon-40b", tp=4, pp=2, vpp_layers=10, seq=2048, mbs=2,
                              nmicro=8, sp=True),
    # config #5 as the reference runs it: every layer recomputed
    "llama70b-tp8": dict(model="llama2-70b", tp=8, pp=1, seq=4096, mbs=2, nmicro=8, sp=True,
                         recompute="full", dist_opt=True),
    # MI355X variant of config #5: 288 GB per GPU holds most or all of the
    # activations, so the memory model picks the recompute depth for a 260 GB peak
    "llama70b-tp8-budget": dict(model="llama2-70b", tp=8, pp=1, seq=4096, mbs=2, nmicro=8,
                                sp=True, recompute_budget_gb=260, dist_opt=True),
    # MI355X addition (no reference counterpart): long-context training with
    # context parallelism, each 32k-token sequence split over 8 GPUs (zig-zag
    # ring attention, parallel/context.py)
    "llama7b-cp8-seq32k": dict(model="llama2-7b", tp=1, pp=1, cp=8, seq=32768, mbs=1, nmicro=8),
}

PROXIES = {  # one TP rank of a BASELINE config on one GPU
    "llama7b-tp8": ("llama7b-tp8-seq4096", 8),
    "llama70b-tp8": ("llama70b-tp8", 8),
    "llama70b-tp8-budget": ("llama70b-tp8-budget", 8),
    "falcon40b-tp4-pp2": ("falcon40b-tp4-pp2", 4),
}


def _parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--preset", default="llama7b-dp", choices=sorted(PRESETS))
    ap.add_argument("--proxy", default=None, choices=sorted(PROXIES))
    ap.add_argument("--model", default=None, choices=sorted(MODELS))
    ap.add_argument("--seq_len", type=int, default=None)
    ap.add_argument("--micro_batch", type=int, default=None)
    ap.add_argument("--num_micro", type=int, default=None, help="micro-batches per step")
    ap.add_argument("--tp", type=int, default=None)
    ap.add_argument("--pp", type=int, default=None)
    ap.add_argument("--cp", type=int, default=None, help="context-parallel size")
    ap.add_argument("--vpp_layers", type=int, default=None,
                    help="layers per virtual pipeline stage (interleaved 1F1B)")
    ap.add_argument("--recompute", default=None, choices=["selective", "full"])
    ap.add_argument("--comm_diag", action="store_true",
                    help="add the per-collective table of one extra timed-collective step "
                         "(always on at --gpus > 1)")
    ap.add_argument("--recompute_budget_gb", type=float, default=None,
                    help="recompute only what the memory model needs to fit this peak")
    ap.add_argument("--no_sp", action="store_true")
    ap.add_argument("--no_dist_opt", action="store_true")
    ap.add_argument("--bucket_mb", type=float, default=512.0)
    ap.add_argument("--data", default="cycle", choices=["cycle", "uniform"])
    ap.add_argument("--xgmi_busbw_gbs", type=float, default=300.0,
                    help="proxies: assumed ring bus bandwidth for the analytic TP comm time")
    ap.add_argument("--extra", default="", help="extra framework flags (space separated)")
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(n, argv):
    """Start n ranks of this script; nothing in this process touches the GPU."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv,
                                      env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in alive:  # one rank failed: the collective peers would hang
                    q.terminate()
        time.sleep(0.2)
    for p in procs:
        p.wait()
    return rc


def _resolve(a, world):
    """Model / parallel config from preset + overrides (+ proxy)."""
    cfg = dict(PRESETS[a.preset])
    proxy_tp = None
    if a.proxy:
        cfg = dict(PRESETS[PROXIES[a.proxy][0]])
        proxy_tp = PROXIES[a.proxy][1]
    for k, v in (("model", a.model), ("seq", a.seq_len), ("mbs", a.micro_batch),
                 ("nmicro", a.num_micro), ("tp", a.tp), ("pp", a.pp), ("cp", a.cp),
                 ("vpp_layers", a.vpp_layers), ("recompute", a.recompute),
                 ("recompute_budget_gb", a.recompute_budget_gb)):
        if v is not None:
            cfg[k] = v
    if a.no_sp:
        cfg["sp"] = False
    shape = dict(MODELS[cfg["model"]])
    if proxy_tp:
        # one TP rank (and one PP stage) of the real model on one GPU: the
        # framework builds TP rank 0 of a TP=proxy_tp model (sharded heads,
        # FFN, vocab; s/tp-row norms / residuals under SP) and its TP
        # collectives loop back locally (--simulated_tensor_parallel_size)
        shape["L"] //= cfg.get("pp", 1)
        cfg.update(sim_tp=proxy_tp, tp=1, pp=1, vpp_layers=None)
    return cfg, shape


def _framework_argv(a, cfg, shape, world, on_gpu):
    tp, pp, cp = cfg.get("tp", 1), cfg.get("pp", 1), cfg.get("cp", 1) or 1
    if world % (tp * pp * cp):
        raise SystemExit(f"--gpus {world} is not a multiple of tp*pp*cp = {tp * pp * cp}")
    dp = world // (tp * pp * cp)  # ranks reading different samples
    mbs, nmicro, seq = cfg["mbs"], cfg["nmicro"], cfg["seq"]
    gbs = mbs * nmicro * dp
    s = shape
    argv = ["--num_layers", str(s["L"]), "--hidden_size", str(s["h"]),
            "--num_attention_heads", str(s["nh"]),
            "--seq_length", str(seq), "--max_position_embeddings", str(max(4096, seq)),
            "--position_embedding_type", "rotary", "--layernorm_epsilon", "1e-5",
            "--hidden_dropout", "0.0", "--attention_dropout", "0.0", "--no_bias_gelu_fusion",
            "--no_bias_dropout_fusion", "--use_flash_attn", "--micro_batch_size", str(mbs),
            "--global_batch_size", str(gbs), "--train_iters", str(a.steps + a.warmup + 2),
            "--lr", "3e-4", "--min_lr", "3e-5", "--lr_decay_style", "cosine",
            "--lr_warmup_iters", "1", "--adam_beta2", "0.95", "--adam_eps", "1e-5",
            "--weight_decay", "0.1", "--clip_grad", "1.0", "--log_interval", "1000000",
            "--eval_interval", "1000000", "--eval_iters", "0", "--tokenizer_type",
            "NullTokenizer", "--synthetic_data", "--synthetic_pattern", a.data,
            "--synthetic_vocab_size", str(s["vocab"]), "--make_vocab_size_divisible_by", "128",
            "--num_workers", "0", "--ddp_bucket_size_mb", str(a.bucket_mb),
            "--tensor_model_parallel_size", str(tp), "--pipeline_model_parallel_size", str(pp),
            "--context_parallel_size", str(cp)]
    if s.get("ffn"):
        argv += ["--ffn_hidden_size", str(s["ffn"])]
    if s.get("nkv"):
        argv += ["--num_attention_heads_kv", str(s["nkv"])]
    if s.get("kv_channels"):
        argv += ["--kv_channels", str(s["kv_channels"])]
    if s["family"] == "llama2":
        argv += ["--use_rms_norm", "--glu_activation", "swiglu", "--no_tie_embed_logits",
                 "--model_name", "llama2"]
    else:
        argv += ["--parallel_attn", "--model_name", "falcon"]
        if s.get("parallel_layernorm"):
            argv += ["--parallel_layernorm"]
    sim_tp = cfg.get("sim_tp")
    if sim_tp:
        argv += ["--simulated_tensor_parallel_size", str(sim_tp)]
    if cfg.get("sp") and (tp > 1 or sim_tp):
        argv += ["--sequence_parallel"]
    if cfg.get("vpp_layers") and pp > 1:
        argv += ["--num_layers_per_virtual_pipeline_stage", str(cfg["vpp_layers"])]
        if pp == 2:
            argv += ["--allow_interleaved_pp2"]
    if on_gpu:
        argv += ["--bf16"]
    else:
        argv += ["--distributed_backend", "gloo"]
    dist_opt = (dp * cp > 1 or cfg.get("dist_opt")) and not a.no_dist_opt
    if dist_opt:
        argv += ["--use_distributed_optimizer"]
    rc = cfg.get("recompute")
    if rc:
        argv += ["--recompute_granularity", rc]
        if rc == "full":
            argv += ["--recompute_method", "uniform", "--recompute_num_layers", "1"]
    elif cfg.get("recompute_budget_gb"):
        rc = f"budget{cfg['recompute_budget_gb']:g}gb"
        argv += ["--recompute_memory_budget_gb", str(cfg["recompute_budget_gb"])]
    if a.extra:
        argv += a.extra.split()
    return argv, dict(tp=tp, pp=pp, cp=cp, dp=dp, gbs=gbs, mbs=mbs, nmicro=nmicro, seq=seq,
                      dist_opt=bool(dist_opt), vpp=cfg.get("vpp_layers") if pp > 1 else None,
                      recompute=rc, sp=bool(cfg.get("sp") and (tp > 1 or sim_tp)),
                      sim_tp=sim_tp)


def _proxy_comm(rep, n, steps, ms_step, busbw_gbs):
    """Per-step TP traffic of the simulated rank (from the comm accounting)
    and an analytic xGMI time for it: ring all-gather / reduce-scatter move
    (n-1)/n of the full buffer per rank, all-reduce twice that, at a bus
    bandwidth of ``busbw_gbs`` GB/s (an assumption, stated in the record)."""
    tp_bytes, wire = 0.0, 0.0
    detail = {}
    for key, (cnt, nbytes, _) in rep.items():
        op, _, grp = key.partition("/")
        if grp != "tp":
            continue
        f = (n - 1) / n * (2.0 if op == "all_reduce" else 1.0)
        tp_bytes += nbytes
        wire += nbytes * f
        detail[op] = {"calls_per_step": cnt / steps, "MiB_per_step": round(nbytes / steps / 2**20, 1)}
    ms = wire / steps / (busbw_gbs * 1e9) * 1e3
    return {"proxy_tp_collectives": detail,
            "proxy_tp_wire_MiB_per_step": round(wire / steps / 2**20, 1),
            "proxy_xgmi_busbw_GBs_assumed": busbw_gbs,
            "proxy_tp_comm_ms_per_step_analytic": round(ms, 2),
            "proxy_ms_per_step_if_comm_not_overlapped": round(ms_step + ms, 2)}


def _comm_diag(rep, step_ms):
    """Per-collective table of one extra (untimed) step with HIP-event timing on:
    calls, bytes, in-flight ms (issue -> wait), algorithm and bus bandwidth
    (ring factors over the group's rank count) — so a multi-GPU record says
    where its time goes without another run (reference: megatron/timers.py:162-203)."""
    from epfl_megatron_amd.parallel import comm
    fac = {"all_reduce": lambda n: 2.0 * (n - 1) / n, "all_gather": lambda n: (n - 1) / n,
           "reduce_scatter": lambda n: (n - 1) / n}
    per, tot = {}, 0.0
    for key, (cnt, nbytes, ms) in rep.items():
        op, _, grp = key.partition("/")
        n = comm.group_size(grp)
        d = {"calls": cnt, "MiB": round(nbytes / 2**20, 1), "ms_in_flight": round(ms, 2)}
        if n:
            d["ranks"] = n
        if ms > 0 and nbytes:
            alg = nbytes / (ms * 1e-3) / 1e9
            d["algbw_GBs"] = round(alg, 1)
            if n and op in fac:
                d["busbw_GBs"] = round(alg * fac[op](n), 1)
        per[key] = d
        tot += ms
    return {"step_ms_with_timing": round(step_ms, 2), "sum_ms_in_flight": round(tot, 2),
            "collectives": per}


def _n1_ref_path(label, par):
    import tempfile
    key = f"{label}_s{par['seq']}_mb{par['mbs']}x{par['nmicro']}_tp{par['tp']}pp{par['pp']}cp{par['cp']}"
    key = "".join(c if c.isalnum() else "_" for c in key)
    return os.path.join(tempfile.gettempdir(), f"ema_bench_n1_{key}.json")


def _label(cfg, shape, a):
    names = {"llama2-7b": "Llama-2-7B", "llama2-13b": "Llama-2-13B", "llama2-70b": "Llama-2-70B",
             "falcon-7b": "Falcon-7B", "falcon-40b": "Falcon-40B"}
    return names.get(cfg["model"], cfg["model"])


def main(argv=None):
    raw = list(sys.argv[1:] if argv is None else argv)
    a = _parse(raw)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(_spawn(a.gpus, raw))

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus={a.gpus}: launch one rank per GPU")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    on_gpu = torch.cuda.is_available()
    cfg, shape = _resolve(a, world)
    if not on_gpu:  # CPU plumbing run (gloo): tiny model of the same family
        fam = shape
        cfg.update(model="tiny", seq=min(cfg["seq"], 128), mbs=2,
                   nmicro=max(2, cfg.get("pp", 1) * 2))
        shape = dict(MODELS["tiny"], family=fam["family"],
                     parallel_layernorm=fam.get("parallel_layernorm", False))
        if fam["family"] == "falcon":
            shape.update(ffn=None, nkv=max(2, cfg.get("tp", 1), cfg.get("sim_tp") or 1))
        if cfg.get("tp", 1) > 1 or cfg.get("pp", 1) > 1 or cfg.get("sim_tp"):
            shape["nh"] = 8
        shape["L"] = max(shape["L"], 2 * cfg.get("pp", 1))
        if cfg.get("vpp_layers"):
            cfg["vpp_layers"] = 1
    fargv, par = _framework_argv(a, cfg, shape, world, on_gpu)

    import finetune
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.initialize import initialize_megatron
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.training import (_setup_model_and_optimizer,
                                            build_train_valid_test_data_iterators, train_step)
    from epfl_megatron_amd.parallel import state
    from epfl_megatron_amd.utils.flops import flops_per_token

    initialize_megatron(finetune.extra_args, {"tokenizer_type": "NullTokenizer"}, args_list=fargv)
    args = get_args()
    chunks, optimizer, sched = _setup_model_and_optimizer(finetune.model_provider,
                                                         ModelType.encoder_or_decoder, args=args)
    if args.virtual_pipeline_model_parallel_size is not None:
        its = [build_train_valid_test_data_iterators(finetune.train_valid_test_datasets_provider,
                                                     args) for _ in chunks]
        train_it = [i[0] for i in its]
    else:
        train_it, _, _ = build_train_valid_test_data_iterators(
            finetune.train_valid_test_datasets_provider, args)
    for m in chunks:
        m.train()

    def sync():
        if on_gpu:
            torch.cuda.synchronize()
        dist.barrier()

    losses = []

    def step():
        out = train_step(finetune.forward_step, train_it, chunks, optimizer, sched, args)
        args.consumed_train_samples += par["gbs"]
        if out[0]:
            losses.append(out[0]["lm loss"])
        return out

    from epfl_megatron_amd.parallel import comm
    for _ in range(a.warmup):
        step()
    sync()
    comm.report(reset=True)
    if on_gpu:
        torch.cuda.reset_peak_memory_stats()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    sync()
    dt = time.perf_counter() - t0
    comm_rep = comm.report(reset=True)
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # slowest rank defines the step time
    dt = float(t.item())
    mem = torch.tensor([torch.cuda.max_memory_allocated() / 2**30 if on_gpu else 0.0],
                       dtype=torch.float64, device=dev)
    dist.all_reduce(mem, op=dist.ReduceOp.MAX)
    # the loss lives on the last pipeline stage: ship it to rank 0
    loss_t = torch.tensor([float(losses[0]) if losses else float("nan"),
                           float(losses[-1]) if losses else float("nan")],
                          dtype=torch.float64, device=dev)
    if state.get_pipeline_model_parallel_world_size() > 1:
        src = state.get_pipeline_model_parallel_last_rank()
        dist.broadcast(loss_t, src=src, group=state.get_pipeline_model_parallel_group())
    diag = None
    if world > 1 or a.comm_diag:
        # one more step, untimed, with per-collective HIP-event timing
        comm.set_timing(True)
        t1 = time.perf_counter()
        step()
        for m in chunks:  # the dist-opt parameter all-gather still in flight
            if hasattr(m, "wait_param_sync"):
                m.wait_param_sync()
        sync()
        diag = _comm_diag(comm.report(reset=True), (time.perf_counter() - t1) * 1e3)
        fargs = get_args()
        diag["model"] = {"layers_per_stage": fargs.num_layers // fargs.pipeline_model_parallel_size,
                         "hidden": fargs.hidden_size,
                         "bytes_per_el": 2 if (fargs.bf16 or fargs.fp16) else 4}
        comm.set_timing(False)
    optimizer.resolve_pending()
    tokens = par["gbs"] * par["seq"] * a.steps
    tok_s = tokens / dt
    # a simulated TP rank processes every token of its TP group at 1/tp of the
    # FLOPs: per-GPU rate of the real configuration = group rate / tp
    per_gpu = tok_s / world / (par["sim_tp"] or 1)
    fpt = flops_per_token(args)
    mfu = per_gpu * fpt / (args.peak_tflops * 1e12)
    if dist.get_rank() == 0:
        parallel = f"dp{par['dp']}"
        if par["sim_tp"]:
            parallel = f"proxy-tp{par['sim_tp']}" + ("+sp" if par["sp"] else "")
        if par["tp"] > 1:
            parallel = f"tp{par['tp']}" + ("+sp" if par["sp"] else "") + \
                (f"_dp{par['dp']}" if par["dp"] > 1 else "")
        if par["cp"] > 1:
            parallel += f"+cp{par['cp']}"
        if par["pp"] > 1:
            parallel += f"_pp{par['pp']}" + (f"+vpp{par['vpp']}" if par["vpp"] else "")
        if par["dist_opt"]:
            parallel += "+distopt"
        if par["recompute"]:
            parallel += f"+recompute_{par['recompute']}"
        label = _label(cfg, shape, a)
        dtype = "bf16" if on_gpu else "fp32"
        if a.proxy:
            metric = (f"PROXY (1 GPU = one TP rank of {a.proxy}; not the BASELINE metric): "
                      f"tokens/s of the TP group this rank belongs to, {dtype} "
                      "(per-GPU = value / tp in 'tokens_per_sec_per_gpu')")
            label = f"{label} [{a.proxy} per-rank proxy]"
        elif cfg["model"] == "llama2-7b":
            metric = (f"{BASELINE_METRIC} [{label} {dtype} training; value = tokens/s aggregate "
                      "over all GPUs, per-GPU = value / n_gpus, MFU in 'mfu']")
        else:  # another BASELINE config: do not claim the Llama-2-7B headline
            metric = (f"tokens/sec/GPU + MFU, {label} {dtype} training, preset {a.preset} "
                      "[value = tokens/s aggregate over all GPUs, MFU in 'mfu'; "
                      "not the headline metric of BASELINE.json]")
        rec = {
            "metric": metric,
            "value": round(tok_s, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * dt / a.steps, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(per_gpu / REF_TOKENS_PER_SEC_PER_GPU, 3)
                            if cfg["model"] == "llama2-7b" and par["seq"] == 1024
                            and not a.proxy else None),
            "dtype": dtype,
            "data": f"synthetic ({a.data} tokens), random-init weights",
            "config": {"model": label, "global_batch": par["gbs"], "seq_len": par["seq"],
                       "micro_batch": par["mbs"], "num_micro_batches": par["nmicro"],
                       "parallelism": parallel},
            "tokens_per_sec_per_gpu": round(per_gpu, 2),
            "mfu": round(mfu, 4),
            "tflops_per_gpu": round(per_gpu * fpt / 1e12, 1),
            "flops_per_token": fpt,
            "peak_tflops_assumed": args.peak_tflops,
            "first_loss": round(float(loss_t[0]), 4),
            "final_loss": round(float(loss_t[1]), 4),
            "max_mem_gb": round(float(mem[0]), 1) if on_gpu else None,
            "backend": dist.get_backend(),
            "world_size": world,
            "dp": par["dp"], "tp": par["tp"], "pp": par["pp"], "cp": par["cp"],
            "recompute": {"granularity": args.recompute_granularity,
                          "method": args.recompute_method,
                          "layers": (args.recompute_num_layers
                                     if args.recompute_granularity == "full" else 0),
                          "estimated_peak_gb": (round(args.recompute_estimate_gb, 1)
                                                if getattr(args, "recompute_estimate_gb", None)
                                                else None)},
        }
        if a.proxy:
            rec.update(_proxy_comm(comm_rep, par["sim_tp"], a.steps, 1000.0 * dt / a.steps,
                                   a.xgmi_busbw_gbs))
        # weak-scaling reference: an N=1 run of the same per-GPU config leaves its
        # step time behind; an N>1 run reports the step time it lost to N ranks
        if not a.proxy and par["dp"] >= 1:
            ref_path = _n1_ref_path(label, par)
            if world == 1 and on_gpu:
                try:
                    with open(ref_path, "w") as f:
                        json.dump({"ms_per_step": rec["ms_per_step"]}, f)
                except OSError:
                    pass
            elif world > 1 and diag is not None and os.path.exists(ref_path):
                try:
                    n1 = json.load(open(ref_path))["ms_per_step"]
                    diag["n1_ms_per_step"] = n1
                    diag["exposed_ms_vs_n1"] = round(rec["ms_per_step"] - n1, 2)
                except (OSError, ValueError, KeyError):
                    pass
        if diag is not None:
            rec["comm_diag"] = diag
        print(json.dumps(rec), flush=True)
    else:
        rec = None
    dist.barrier()
    dist.destroy_process_group()
    return rec


if __name__ == "__main__":
    main()

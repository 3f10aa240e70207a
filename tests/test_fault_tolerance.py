"""Preemption: SIGTERM mid-run -> checkpoint -> resume == uninterrupted run
(reference ``megatron/dist_signal_handler.py:50-81`` and
``megatron/training.py:712-718``).

Two ranks under torchrun (gloo).  SIGTERM goes to ONE rank only, at a random
point of the run; the all-gathered flag makes both ranks checkpoint the same
iteration and exit cleanly.  Resuming from that checkpoint and training to the
end must give bit-identical final weights to a run that was never
interrupted, wherever the signal landed.
"""
import os
import signal
import subprocess
import sys
import time

import psutil
import torch

from dist_utils import TINY_LLAMA, free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ITERS = 14


def _cmd(save, load=None, extra=()):
    argv = [a for a in TINY_LLAMA]
    argv[argv.index("--train_iters") + 1] = str(ITERS)
    argv[argv.index("--log_interval") + 1] = "1"
    argv += ["--micro_batch_size", "1", "--global_batch_size", "4", "--save", save,
             "--save_interval", "1000", "--distributed_backend", "gloo", "--num_workers", "0",
             "--exit_signal_handler"] + list(extra)
    if load:
        argv += ["--load", load]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
            os.path.join(ROOT, "finetune.py")] + argv


def _env():
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    return env


def _final_weights(ckdir):
    from epfl_megatron_amd.checkpointing import safe_load
    it = open(os.path.join(ckdir, "latest_checkpointed_iteration.txt")).read().strip()
    sd = safe_load(os.path.join(ckdir, f"iter_{int(it):07d}", "mp_rank_00", "model_optim_rng.pt"))
    return int(it), sd["model"]


def _flat(d, prefix=""):
    out = {}
    for k, v in d.items():
        if isinstance(v, dict):
            out.update(_flat(v, prefix + k + "."))
        elif torch.is_tensor(v):
            out[prefix + k] = v
    return out


def test_sigterm_checkpoint_and_resume_is_exact(tmp_path):
    straight = str(tmp_path / "straight")
    r = subprocess.run(_cmd(straight), cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]

    pre = str(tmp_path / "pre")
    p = subprocess.Popen(_cmd(pre), cwd=ROOT, env=_env(), stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, text=True)
    killed_at = None
    try:
        for line in p.stdout:
            if " iteration " in line and f"/{ITERS:8d}" in line:
                it = int(line.split(" iteration ")[1].split("/")[0])
                if it >= 3 and killed_at is None:
                    kids = psutil.Process(p.pid).children(recursive=True)
                    workers = [k for k in kids if "finetune.py" in " ".join(k.cmdline())]
                    assert len(workers) == 2, [k.cmdline() for k in kids]
                    os.kill(max(w.pid for w in workers), signal.SIGTERM)  # one rank only
                    killed_at = it
        rc = p.wait(timeout=300)
    finally:
        if p.poll() is None:
            p.kill()
    assert killed_at is not None
    assert rc == 0
    saved_it, _ = _final_weights(pre)
    assert killed_at <= saved_it < ITERS  # both ranks stopped at the same, early iteration

    r = subprocess.run(_cmd(pre, load=pre), cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    it_a, wa = _final_weights(straight)
    it_b, wb = _final_weights(pre)
    assert it_a == it_b == ITERS
    fa, fb = _flat(wa), _flat(wb)
    assert fa.keys() == fb.keys()
    for k in fa:
        assert torch.equal(fa[k], fb[k]), k

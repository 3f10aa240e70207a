"""bench.py driver contract on the CPU/gloo path: ``--gpus N`` without torchrun
spawns N ranks itself and reports n_gpus = N."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=600):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                         env=env, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-3000:]
    return json.loads(lines[0])


def test_bench_spawns_ranks():
    rec = _run(["--gpus", "4", "--steps", "1", "--warmup", "1"])
    assert rec["n_gpus"] == 4
    assert rec["config"]["parallelism"] == "dp4+distopt"
    assert rec["config"]["global_batch"] == 4 * rec["config"]["micro_batch"] * \
        rec["config"]["num_micro_batches"]
    for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in rec
    assert rec["value"] > 0 and rec["scaling"] == "weak"


def test_bench_single_rank_default():
    rec = _run(["--steps", "2", "--warmup", "1"])
    assert rec["n_gpus"] == 1 and rec["config"]["parallelism"] == "dp1"


def test_bench_rank_failure_propagates():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--steps", "1", "--warmup", "0", "--tp", "3"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode != 0

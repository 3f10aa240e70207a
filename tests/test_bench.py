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
    # self-diagnosing multi-rank record: per-collective
    # counts, bytes, in-flight time and bandwidth of one extra timed step
    diag = rec["comm_diag"]
    assert diag["step_ms_with_timing"] > 0 and diag["sum_ms_in_flight"] > 0
    rs = [v for k, v in diag["collectives"].items() if k.startswith("reduce_scatter/dp")]
    ag = [v for k, v in diag["collectives"].items() if k.startswith("all_gather/dp")]
    assert rs and ag, diag["collectives"].keys()
    for d in rs + ag:
        assert d["calls"] > 0 and d["MiB"] > 0 and d["ranks"] == 4
        assert d["ms_in_flight"] > 0 and d["busbw_GBs"] > 0


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


def test_bench_labels_follow_dtype_and_model():
    """The metric names the real compute dtype, non-7B presets do not carry
    the Llama-2-7B headline metric, and the record names the backend and the
    parallel group sizes."""
    rec = _run(["--steps", "1", "--warmup", "0"])
    assert rec["dtype"] == "fp32" and "bf16" not in rec["metric"]
    assert rec["backend"] == "gloo" and rec["world_size"] == 1
    assert (rec["dp"], rec["tp"], rec["pp"]) == (1, 1, 1)
    rec = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--preset", "falcon40b-tp4-pp2",
                "--tp", "1", "--pp", "2"])
    assert "Llama-2 7B" not in rec["metric"] and "Llama-2-7B" not in rec["metric"]
    assert rec["pp"] == 2 and rec["world_size"] == 2


def test_readme_headline_quotes_driver_record():
    """README's headline number is the driver's own BENCH_r*.json value."""
    import re
    readme = open(os.path.join(ROOT, "README.md")).read()
    row = next(l for l in readme.splitlines() if "(headline" in l and l.startswith("|"))
    m = re.search(r"\*\*([0-9.]+)k\*\* \(driver run, `(BENCH_r\d+\.json)`\)", row)
    assert m, row
    rec = json.load(open(os.path.join(ROOT, m.group(2))))
    value = rec["parsed"]["value"] if "parsed" in rec else rec["value"]
    assert abs(float(m.group(1)) - value / 1000) < 0.051, (m.group(1), value)


import pytest  # noqa: E402


@pytest.mark.parametrize("preset,parallel,groups", [
    ("llama7b-tp8-seq4096", "tp8+sp", (1, 8, 1)),
    ("falcon40b-tp4-pp2", "tp4+sp_pp2+vpp1", (1, 4, 2)),
    ("llama70b-tp8", "tp8+sp+distopt+recompute_full", (1, 8, 1)),
])
def test_bench_multi_gpu_presets_on_gloo(preset, parallel, groups):
    """The three multi-GPU BASELINE presets run end to end at 8 ranks (the
    driver's 8-GPU layout) through the same code RCCL runs, incl. the startup
    collective self-check."""
    rec = _run(["--gpus", "8", "--preset", preset, "--steps", "1", "--warmup", "1"], timeout=900)
    assert rec["n_gpus"] == 8 and rec["config"]["parallelism"] == parallel
    assert (rec["dp"], rec["tp"], rec["pp"]) == groups
    assert rec["value"] > 0 and rec["final_loss"] == rec["final_loss"]  # not NaN


def test_llama70b_presets_keep_the_reference_recompute():
    """BASELINE config #5 recomputes every layer; the memory-model
    policy is a separately labelled preset."""
    import bench
    for preset, rc, flag in (("llama70b-tp8", "full", "--recompute_granularity"),
                             ("llama70b-tp8-budget", "budget260gb",
                              "--recompute_memory_budget_gb")):
        a = bench._parse(["--preset", preset])
        cfg, shape = bench._resolve(a, 8)
        argv, par = bench._framework_argv(a, cfg, shape, 8, on_gpu=False)
        assert par["recompute"] == rc and flag in argv


def test_proxy_is_one_simulated_tp_rank():
    """--proxy builds TP rank 0 of the real model (--simulated_tensor_parallel_size):
    sequence parallel is on, the TP collectives run as local loopbacks and are
    reported per step with an analytic xGMI time."""
    rec = _run(["--proxy", "llama7b-tp8", "--steps", "1", "--warmup", "1"])
    assert rec["config"]["parallelism"] == "proxy-tp8+sp"
    assert "PROXY" in rec["metric"]
    coll = rec["proxy_tp_collectives"]
    # per layer: all-gathers before qkv and fc1, reduce-scatters after o-proj and fc2
    assert coll["all_gather"]["calls_per_step"] > 0 and coll["reduce_scatter"]["calls_per_step"] > 0
    assert rec["proxy_tp_comm_ms_per_step_analytic"] > 0
    assert rec["tokens_per_sec_per_gpu"] * 8 == pytest.approx(rec["value"], rel=1e-3)


def test_bench_context_parallel_preset_on_gloo():
    """--preset llama7b-cp8-seq32k scaled down (tiny model, seq 256, CP=2 at 4
    ranks): 2 sample-parallel ranks x 2 sequence chunks, dist-opt over all 4."""
    rec = _run(["--gpus", "4", "--preset", "llama7b-cp8-seq32k", "--cp", "2", "--model", "tiny",
                "--seq_len", "256", "--num_micro", "2", "--steps", "1", "--warmup", "1"])
    assert rec["config"]["parallelism"] == "dp2+cp2+distopt"
    assert (rec["dp"], rec["cp"]) == (2, 2)
    assert rec["config"]["global_batch"] == 2 * 2 * rec["config"]["micro_batch"]
    assert rec["value"] > 0 and rec["final_loss"] == rec["final_loss"]

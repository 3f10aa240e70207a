"""Every BASELINE multi-GPU preset at 8 ranks on gloo, with the in-flight
race checker on (the first RCCL N>1 run must land
cleanly).  bench.py swaps in a tiny model of the same family on CPU (same
TP / PP / VPP / SP / CP / dist-opt / recompute structure, heads and FFN
divisible by TP); the record must carry the per-collective diagnosis table
with the collectives the structure implies."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench8(preset):
    env = dict(os.environ, EMA_COMM_CHECK="1", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8",
                          "--steps", "1", "--warmup", "1", "--preset", preset],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-3000:]
    return json.loads(lines[0])


# preset -> (tp, pp, collective keys that must appear)
CASES = {
    "llama7b-dp": (1, 1, ("reduce_scatter/dp", "all_gather/dp")),
    "llama7b-tp8-seq4096": (8, 1, ("all_gather/tp", "reduce_scatter/tp")),
    "falcon40b-tp4-pp2": (4, 2, ("all_gather/tp", "reduce_scatter/tp", "p2p_send/pp", "p2p_recv/pp")),
    "llama70b-tp8": (8, 1, ("all_gather/tp", "reduce_scatter/tp")),
}


@pytest.mark.parametrize("preset", sorted(CASES))
def test_preset_8_ranks_gloo_race_checked(preset):
    tp, pp, keys = CASES[preset]
    rec = _bench8(preset)
    assert rec["n_gpus"] == 8 and rec["world_size"] == 8
    assert (rec["tp"], rec["pp"]) == (tp, pp) and rec["dp"] == 8 // (tp * pp)
    assert rec["value"] > 0
    coll = rec["comm_diag"]["collectives"]
    for k in keys:
        hits = [c for c in coll if c.startswith(k)]
        assert hits, (k, sorted(coll))
        for c in hits:
            assert coll[c]["calls"] > 0 and coll[c]["MiB"] >= 0

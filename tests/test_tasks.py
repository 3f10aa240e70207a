"""Zero-shot task evaluation (reference tasks/zeroshot_gpt): window logic,
detokenizers, and WikiText loss / LAMBADA accuracy that (a) match a direct
computation with the model and (b) are identical under TP / PP / DP."""
import json
import math
import os
import sys

import numpy as np
import pytest
import torch

from dist_utils import run_dist, init_framework, TINY_LLAMA

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tasks.zeroshot_gpt.datasets import LMDataset  # noqa: E402
from tasks.zeroshot_gpt.detokenizer import get_detokenizer  # noqa: E402


@pytest.mark.parametrize("n,seq,stride", [(100, 16, 4), (100, 16, 16), (17, 16, 4), (5, 16, 4),
                                          (61, 8, 3)])
def test_lm_windows_score_every_target_once(n, seq, stride):
    ds = LMDataset(list(range(n)), seq, 0, n, n, stride)
    seen = []
    for i in range(len(ds)):
        d = ds[i]
        assert d["text"].shape == (seq + 1,) and d["pad_mask"].shape == (seq,)
        start = i * ds.stride
        for pos in np.nonzero(d["pad_mask"])[0]:
            assert d["text"][pos + 1] == start + pos + 1
            seen.append(start + pos + 1)
    assert sorted(seen) == list(range(1, n))


def test_detokenizers():
    wiki = get_detokenizer("wiki.test.tokens")
    assert wiki("the 1 @,@ 000 @-@ year war ( 1914 ) , ended .") == \
        "the 1,000-year war (1914), ended ."
    assert wiki(" = = Heading = = \n") == " == Heading ==\n"
    assert get_detokenizer("ptb.test.txt")("do n't pay $ 1 now") == "don't pay $1 now"
    assert get_detokenizer("lambada_test.jsonl")("as is") == "as is"


def _write_data(tmp):
    rng = np.random.RandomState(0)
    wiki = os.path.join(tmp, "wiki.txt")
    with open(wiki, "w") as f:
        f.write(" ".join(str(x) for x in rng.randint(0, 240, size=75)))
    lam = os.path.join(tmp, "lambada.jsonl")
    with open(lam, "w") as f:
        for k in range(7):
            n = 4 + k * 3  # the last sample is longer than seq_length (kept right-aligned)
            f.write(json.dumps({"text": " ".join(str(x) for x in rng.randint(0, 240, n))}) + "\n")
    return wiki, lam


def _argv(task, path, extra):
    a = [x for x in TINY_LLAMA if x != "--synthetic_data"]
    return a + ["--task", task, "--valid_data", path, "--micro_batch_size", "2",
                "--overlapping_eval", "4",
                "--strict_lambada"] + list(extra)


def _eval(rank, world, task, path, extra):
    import tasks.main as tm
    init_framework(_argv(task, path, extra), tm.get_tasks_args)
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.training import get_model
    from test_parallel_equivalence import _deterministic_init
    from epfl_megatron_amd import get_args
    from tasks.zeroshot_gpt import evaluate as ev
    from tasks.zeroshot_gpt.datasets import build_dataset
    metric = {"LAMBADA": "accuracy", "WIKITEXT103": "loss"}[task]
    model = get_model(ev._model_provider(metric), ModelType.encoder_or_decoder,
                      wrap_with_ddp=False)
    _deterministic_init(model, get_args())
    ds = build_dataset(task)
    res = ev.evaluate_and_print_results(task, ds, model[0], metric)
    if world == 1:  # direct computation for cross-checking
        with torch.no_grad():
            m = model[0].eval()
            direct = 0.0
            for i in range(len(ds)):
                d = ds[i]
                toks = torch.as_tensor(d["text"])[None]
                logits = m(toks[:, :-1], None, None).float()[0]
                mask = torch.as_tensor(d["pad_mask"]).bool()
                tgt = toks[0, 1:]
                if metric == "loss":
                    lp = torch.log_softmax(logits, -1).gather(-1, tgt[:, None])[:, 0]
                    direct += float(-(lp[mask]).sum())
                else:
                    direct += float(bool((logits.argmax(-1) == tgt)[mask].all()))
        res["direct"] = direct
    return res


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    return _write_data(str(tmp_path_factory.mktemp("tasks")))


@pytest.mark.parametrize("task", ["WIKITEXT103", "LAMBADA"])
def test_zeroshot_matches_direct_and_parallel(task, data):
    path = data[0] if task == "WIKITEXT103" else data[1]
    base = run_dist(_eval, 1, task, path, [])[0]
    if task == "WIKITEXT103":
        n_tok = 75
        assert base["loss"] == pytest.approx(base["direct"] / (n_tok - 1), rel=1e-5)
        assert base["ppl"] == pytest.approx(math.exp(base["loss"]), rel=1e-6)
        assert base["token_ratio"] == 1.0
    else:
        assert base["total"] == 7
        assert base["correct"] == base["direct"]
    for world, extra in [(2, ["--tensor_model_parallel_size", "2"]),
                         (2, ["--pipeline_model_parallel_size", "2"]),
                         (2, [])]:
        res = run_dist(_eval, world, task, path, extra)
        got = [r for r in res if r]
        assert len(got) >= 1
        for r in got:
            key = "loss" if task == "WIKITEXT103" else "accuracy"
            assert r[key] == pytest.approx(base[key], rel=1e-5, abs=1e-7)

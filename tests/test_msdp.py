"""Multi-stage dialogue prompting (tasks/msdp): metrics, WoW/WoI processing,
prompt selection and prompt construction (CPU).

The reference has no tests for this task; WoW/WoI data are not in the image,
so synthetic dialogues with the same JSON layout are used and expected outputs
are worked out by hand from the reference's rules (parity unpinned beyond that).
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tasks.msdp import preprocessing as pre  # noqa: E402
from tasks.msdp.evaluate import evaluate_f1  # noqa: E402
from tasks.msdp.metrics import F1Metric, normalize_answer, word_tokenize  # noqa: E402
from tasks.msdp.prompt import build_input, postprocess, read_prompts, run_prompting  # noqa: E402


def test_word_tokenize():
    assert word_tokenize("I don't like it, do you?") == \
        ["I", "do", "n't", "like", "it", ",", "do", "you", "?"]
    assert word_tokenize("She's 3.5 m tall.") == ["She", "'s", "3.5", "m", "tall", "."]


def test_f1_metric():
    assert normalize_answer("The Cat, sat!") == "cat sat"
    p, r, f = F1Metric.compute_each_pair("the cat sat on a mat", "cat on mat today")
    # guess tokens: cat sat on mat (4); gold: cat on mat today (4); common 3
    assert p == pytest.approx(0.75) and r == pytest.approx(0.75) and f == pytest.approx(0.75)
    assert F1Metric.compute_each_pair("", "x") == (0.0, 0.0, 0.0)
    assert F1Metric.compute_each_pair("x", "") == (None, None, None)
    p, r, f = F1Metric.compute_all_pairs(["x b", "c", "q"], ["b c", "", "q"])
    assert f == pytest.approx((0.5 + 1.0) / 2)


def test_evaluate_f1_files(tmp_path):
    g, a = tmp_path / "g.txt", tmp_path / "a.txt"
    g.write_text("paris is big<|endoftext|>\nwhatever\n")
    a.write_text("paris is big\nno_passages_used\n")
    p, r, f = evaluate_f1(str(g), str(a))
    assert (p, r, f) == (1.0, 1.0, 1.0)


WOW = [{
    "chosen_topic": "Cats",
    "dialog": [
        {"speaker": "0_Apprentice", "text": "I love cats"},
        {"speaker": "1_Wizard", "text": "Cats are small carnivores!",
         "checked_sentence": {"s": "The cat is a small carnivorous mammal."},
         "checked_passage": {"p": "Cat"}},
        {"speaker": "0_Apprentice", "text": "Do they sleep a lot?"},
        {"speaker": "1_Wizard", "text": "Yes they do",
         "checked_sentence": {}, "checked_passage": {}},
    ]}]


def test_process_wow(tmp_path):
    raw = tmp_path / "wow.json"
    raw.write_text(json.dumps(WOW))
    out, kn, rs = tmp_path / "p.tsv", tmp_path / "k.txt", tmp_path / "r.txt"
    pre.process_wow_dataset(str(raw), str(out), str(kn), str(rs))
    rows = [line.split("\t") for line in out.read_text().splitlines()]
    assert rows == [
        ["Cat", "I love cats.", "The cat is a small carnivorous mammal.",
         "Cats are small carnivores!"],
        ["Cats", "I love cats. [SEP] Cats are small carnivores! [SEP] Do they sleep a lot?",
         "no_passages_used", "Yes they do."],
    ]
    assert kn.read_text().splitlines()[1] == "no_passages_used"
    assert rs.read_text().splitlines()[0] == "Cats are small carnivores !"


def test_process_woi(tmp_path):
    dialog = {"id1": {"dialog_history": [
        {"action": "Wizard => Apprentice", "text": "Hi there"},
        {"action": "Apprentice => Wizard", "text": "Tell me about\tMars"},
        {"action": "Wizard => SearchAgent", "text": "mars planet"},
        {"action": "SearchAgent => Wizard", "text": ""},
        {"action": "Wizard => Apprentice", "text": "Mars is red.",
         "context": {"contents": [{"content": ["a", "b"]}, {"content": ["Mars is the 4th planet", "c"]}],
                     "selected_contents": [[False], [False, False], [True, False]]}},
        {"action": "Apprentice => Wizard", "text": "cool"},
        {"action": "Wizard => Apprentice", "text": "Bye",
         "context": {"contents": [{"content": ["x"]}],
                     "selected_contents": [[True], [False]]}},
    ]}}
    raw = tmp_path / "woi.jsonl"
    raw.write_text(json.dumps(dialog) + "\n")
    out = tmp_path / "p.tsv"
    pre.process_woi_dataset(str(raw), str(out))
    rows = [line.split("\t") for line in out.read_text().splitlines()]
    assert rows == [["mars planet", "Hi there [SEP] Tell me aboutMars", "Mars is the 4th planet",
                     "Mars is red."]]


def _tsv(path, rows):
    path.write_text("".join("\t".join(r) + "\n" for r in rows))
    return str(path)


def test_knowledge_prompt_selection(tmp_path):
    train = _tsv(tmp_path / "train.tsv", [
        ["Cat", "hello [SEP] do cats purr", "Cat purring is a sound", "r"],
        ["Cat", "hi [SEP] what do cats eat", "Cat food is meat", "r"],
        ["Dog", "dogs bark loudly", "Dog barking is loud", "r"],
        ["Fish", "fish swim", "Fish live in water", "r"],
        ["Fish", "x", "no_passages_used", "r"],
    ])
    test = _tsv(tmp_path / "test.tsv", [
        ["Cat", "tell me [SEP] what do cats eat", "k", "r"],
        ["Dogs", "why do dogs bark loudly", "k", "r"],
    ])
    db = pre.get_database(test, train, "wow_seen")
    assert db[0]["Cat"] == ["( do cats purr ) Cat => Cat purring is a sound",
                            "( what do cats eat ) Cat => Cat food is meat"]
    assert len(db[2]) == 4
    out = tmp_path / "prompts.jsonl"
    pre.prompt_selection_for_knowledge_generation(test, train, "hash", str(out), "wow_seen")
    got = [json.loads(line) for line in out.read_text().splitlines()]
    # seen topic: both Cat examples, the closer dialogue ("what do cats eat") last
    assert got[0] == {"Cat what do cats eat": ["( do cats purr ) Cat => Cat purring is a sound",
                                               "( what do cats eat ) Cat => Cat food is meat"]}
    # unseen topic: one example per distinct training topic, most similar (Dog) last
    ex = got[1]["Dogs why do dogs bark loudly"]
    assert len(ex) == 3 and ex[-1] == "( dogs bark loudly ) Dog => Dog barking is loud"


def test_response_prompt_selection_and_prepare(tmp_path):
    k = "the quick brown fox jumps over the lazy dog near the river bank"
    good = ["T", "hi [SEP] tell me", k, "well the quick brown fox jumps over the lazy dog near the river ok"]
    bad = ["T", "hi", k, "no overlap here at all"]
    train = _tsv(tmp_path / "train.tsv", [good, bad, ["T", "c", "no_passages_used", "x"]])
    out = tmp_path / "resp_prompts.txt"
    ex = pre.prompt_selection_for_response_generation(train, str(out), 1234)
    assert ex == ["Topic: T. User says: tell me We know that: " + k + " System replies: " + good[3]]
    test = _tsv(tmp_path / "test.tsv", [["T", "c1", "gold", "r1"], ["U", "c2", "gold", "r2"]])
    kg = tmp_path / "kg.txt"
    kg.write_text("gen one<|endoftext|>\ngen two\n")
    proc = tmp_path / "proc.tsv"
    pre.prepare_input_for_response_generation(test, str(kg), str(proc))
    assert proc.read_text().splitlines() == ["T\tc1\tgen one\tr1", "U\tc2\tgen two\tr2"]


def test_prompt_construction_and_loop(tmp_path):
    kp = tmp_path / "k.jsonl"
    kp.write_text(json.dumps({"Cat what now": ["ex1 ", "ex2"]}) + "\n"
                  + json.dumps({"Cat what now": ["ignored"]}) + "\n")
    prompts = read_prompts(str(kp), "knowledge", 10)
    assert prompts == {"Cat what now": "ex1 \nex2 \n"}
    line = "Cat\ta [SEP] what now\tk\tr"
    assert build_input(line, "knowledge", prompts) == "ex1 \nex2 \n( what now ) Cat =>"
    rp = tmp_path / "r.txt"
    rp.write_text("p1\np2\np3\n")
    rprompt = read_prompts(str(rp), "response", 2)
    assert build_input("Cat\ta [SEP] isn't it?\tCats purr.\tr", "response", rprompt) == \
        "p1 \np2 \nTopic: Cat. User says: is n't it ? We know that: Cats purr . System replies:"
    assert postprocess("abc", "abc  gen line\nmore") == "gen line"
    calls = []

    def fake(batch):
        calls.append(len(batch))
        return [p + " out" + str(len(p)) + "\nnext" for p in batch]

    outs = run_prompting([line] * 3, "knowledge", prompts, fake, batch_size=2)
    assert calls == [2, 1] and outs == ["out" + str(len(build_input(line, "knowledge", prompts)))] * 3

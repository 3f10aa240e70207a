"""MSDP data preparation (reference ``tasks/msdp/preprocessing.py``).

    python tasks/msdp/preprocessing.py --func {process_wow_dataset,process_woi_dataset,
        get_knwl_gen_prompts,get_resp_gen_prompts,prepare_input} ...

Processed format, one dialogue turn per line:
``topic \\t context (turns joined by " [SEP] ") \\t golden knowledge \\t golden response``.

Prompt selection for knowledge generation ranks training dialogues by the dot
product of query / example embeddings (reference :323-459).  The reference
``torch.load``s a pickled DPR question encoder; here ``--model_file`` is either
a local Hugging Face DPR question-encoder directory (safetensors, loaded with
``from_pretrained``; no pickles are executed) or ``hash`` — a deterministic
hashed unigram+bigram embedding that needs no weights.  Embeddings of all
training dialogues are computed once and scored with one GEMM per query on the
GPU when there is one.

Deliberate difference: for test topics absent from training, the reference
sorts similarities ascending and so picks the 10 *least* similar dialogues
(reference :417-431); we take the 10 most similar (distinct topics), ordered
most-similar last as in the seen-topic branch.
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np
import torch

if __package__ in (None, ""):
    sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
    from tasks.msdp.metrics import word_tokenize
else:
    from .metrics import word_tokenize

NO_KNOWLEDGE = "no_passages_used"


def _clean(s):
    return s.replace("\n", "").replace("\r", "").replace("\t", "")


class _Writers:
    def __init__(self, processed, knwl_ref, resp_ref):
        self.files = [open(p, "w") if p else None for p in (processed, knwl_ref, resp_ref)]

    def write(self, topic, context, knowledge, response):
        proc, fk, fr = self.files
        proc.write("\t".join((topic, context, knowledge, response)) + "\n")
        if fk:
            fk.write(knowledge + "\n")
        if fr:
            fr.write(" ".join(word_tokenize(response)) + "\n")

    def close(self):
        for f in self.files:
            if f:
                f.close()


def process_wow_dataset(raw_file, processed_file, knwl_ref_file=None, resp_ref_file=None):
    """Wizard of Wikipedia JSON -> processed TSV (reference :42-125): one line
    per wizard turn; topic is the checked passage (else the chosen topic)."""
    with open(raw_file) as f:
        dialogs = json.load(f)
    out = _Writers(processed_file, knwl_ref_file, resp_ref_file)
    for sample in dialogs:
        history = []
        for j, turn in enumerate(sample["dialog"]):
            text = turn["text"]
            if not text.endswith(("?", ".", "!")):
                text += "."
            if j == 0:
                history.append(text)
                continue
            speaker = turn["speaker"].lower()
            if "wizard" not in speaker:
                assert "apprentice" in speaker, speaker
                history.append(text)
                continue
            sentences = list(turn["checked_sentence"].values())
            passages = list(turn["checked_passage"].values())
            assert len(sentences) <= 1
            knowledge = sentences[0] if sentences else NO_KNOWLEDGE
            passage = passages[0] if len(passages) == 1 else NO_KNOWLEDGE
            topic = passage if passage != NO_KNOWLEDGE else sample["chosen_topic"]
            out.write(topic, " [SEP] ".join(history), knowledge, text)
            history.append(text)
    out.close()


def process_woi_dataset(raw_file, processed_file, knwl_ref_file=None, resp_ref_file=None):
    """Wizard of Internet JSONL -> processed TSV (reference :128-240): the last
    search query is the topic; turns without selected knowledge are dropped
    from the output but stay in the history."""
    out = _Writers(processed_file, knwl_ref_file, resp_ref_file)
    with open(raw_file) as f:
        for line in f:
            if not line.strip():
                continue
            item = next(iter(json.loads(line).values()))
            history, search = [], ""
            for turn in item["dialog_history"]:
                action = turn["action"]
                if action == "Wizard => SearchAgent":
                    search = turn["text"]
                elif action == "Apprentice => Wizard":
                    history.append(turn["text"])
                elif action == "Wizard => Apprentice":
                    if not history:
                        history.append(turn["text"])
                        continue
                    contents = turn["context"]["contents"]
                    selects = turn["context"]["selected_contents"]
                    none_used, selects = selects[0][0], selects[1:]
                    assert len(selects) == len(contents)
                    knowledge = ""
                    if not none_used:
                        # first selected sentence of the LAST document with a
                        # selection (the reference's break leaves only the inner loop)
                        for content, sel in zip(contents, selects):
                            content = content["content"]
                            assert len(content) == len(sel)
                            hit = next((c for c, s in zip(content, sel) if s), None)
                            if hit is not None:
                                knowledge = hit
                    topic = search if (knowledge and not none_used) else "no_topic"
                    response = _clean(turn["text"])
                    if topic != "no_topic":
                        out.write(_clean(topic), _clean(" [SEP] ".join(history)),
                                  _clean(knowledge), response)
                    history.append(response)
                else:
                    assert action == "SearchAgent => Wizard", \
                        "Please check whether you have used the correct data!"
    out.close()


def _read_tsv(path):
    with open(path) as f:
        return [line.rstrip("\n").split("\t") for line in f if line.strip()]


def _dialog_query(topic, turns, with_topic):
    return ("( " + topic + " ) " if with_topic else "") + " ".join(turns)


def get_database(test_datapath, train_datapath, data_type):
    """-> (examples by test topic, dialogues by test topic, all (topic, dialogue,
    example) triples) from the training TSV (reference :243-320)."""
    assert data_type in ("wow_seen", "wow_unseen", "woi"), "Please input a correct data type!!"
    test_topics = {row[0] for row in _read_tsv(test_datapath)}
    by_topic, dialogs_by_topic, examples = {}, {}, []
    strict = data_type != "wow_seen"
    for row in _read_tsv(train_datapath):
        topic, turns, knowledge = row[0], row[1].split(" [SEP] ")[-3:], row[2]
        if knowledge == NO_KNOWLEDGE:
            continue
        if strict and ("(" in knowledge or ")" in knowledge or topic not in knowledge):
            continue
        instance = "( " + turns[-1] + " ) " + topic + " => " + knowledge
        dialog = _dialog_query(topic, turns, strict)
        if topic in test_topics:
            by_topic.setdefault(topic, []).append(instance)
            dialogs_by_topic.setdefault(topic, []).append(dialog)
        elif len(knowledge.split()) > 20 or knowledge.startswith(("It", "it", "This", "this")):
            continue
        examples.append((topic, dialog, instance))
    return by_topic, dialogs_by_topic, examples


class HashEncoder:
    """Weight-free sentence embedding: signed feature hashing of lower-cased
    unigrams and bigrams, L2-normalised."""

    def __init__(self, dim=4096):
        self.dim = dim

    def _feats(self, text):
        toks = [t.lower() for t in word_tokenize(text)]
        return toks + [a + " " + b for a, b in zip(toks, toks[1:])]

    def __call__(self, texts):
        out = np.zeros((len(texts), self.dim), dtype=np.float32)
        for i, t in enumerate(texts):
            for f in self._feats(t):
                h = int.from_bytes(hashlib.blake2b(f.encode(), digest_size=8).digest(), "little")
                out[i, h % self.dim] += 1.0 if (h >> 63) & 1 else -1.0
        n = np.linalg.norm(out, axis=1, keepdims=True)
        return torch.from_numpy(out / np.maximum(n, 1e-12))


class DPREncoder:
    """Local Hugging Face DPR question encoder (``pooler_output`` embeddings)."""

    def __init__(self, path, device):
        from transformers import DPRQuestionEncoder, DPRQuestionEncoderTokenizer
        self.tok = DPRQuestionEncoderTokenizer.from_pretrained(path, local_files_only=True)
        self.model = DPRQuestionEncoder.from_pretrained(
            path, local_files_only=True, use_safetensors=True).to(device).eval()
        self.device = device

    @torch.no_grad()
    def __call__(self, texts, batch=64):
        outs = []
        for i in range(0, len(texts), batch):
            enc = self.tok(texts[i:i + batch], padding=True, truncation=True,
                           return_tensors="pt").to(self.device)
            outs.append(self.model(**enc).pooler_output.float().cpu())
        return torch.cat(outs)


def load_encoder(model_file):
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    if model_file in (None, "", "hash"):
        return HashEncoder()
    return DPREncoder(model_file, dev)


def select_knowledge_prompts(test_rows, database, encoder, data_type, max_examples=10):
    """One ``{"<topic> <last turn>": [examples]}`` per test row (most similar last)."""
    by_topic, dialogs_by_topic, examples = database
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    all_emb = encoder([e[1] for e in examples]).to(dev) if examples else None
    topic_emb = {}
    out = []
    for row in test_rows:
        topic, turns = row[0], row[1].split(" [SEP] ")[-3:]
        query = encoder([_dialog_query(topic, turns, data_type != "wow_seen")]).to(dev)[0]
        if topic in by_topic:
            if topic not in topic_emb:
                topic_emb[topic] = encoder(dialogs_by_topic[topic]).to(dev)
            sims = topic_emb[topic] @ query
            k = min(len(by_topic[topic]), max_examples)
            idx = torch.topk(sims, k).indices.tolist()[::-1]
            chosen = [by_topic[topic][i] for i in idx]
        else:
            order = torch.argsort(all_emb @ query, descending=True).tolist()
            seen, chosen = set(), []
            for i in order:
                t = examples[i][0]
                if t not in seen:
                    seen.add(t)
                    chosen.append(examples[i][2])
                    if len(chosen) == max_examples:
                        break
            chosen = chosen[::-1]
        out.append({topic + " " + turns[-1]: chosen})
    return out


def prompt_selection_for_knowledge_generation(test_datapath, train_datapath, model_path,
                                              output_prompt_path, data_type):
    database = get_database(test_datapath, train_datapath, data_type)
    prompts = select_knowledge_prompts(_read_tsv(test_datapath), database,
                                       load_encoder(model_path), data_type)
    with open(output_prompt_path, "w") as f:
        for p in prompts:
            f.write(json.dumps(p) + "\n")


def _overlap_tokens(knowledge_toks, response_toks, min_run=10):
    """Tokens of ``response`` inside runs of >= ``min_run`` consecutive tokens
    that all occur in the knowledge sentence."""
    vocab = set(knowledge_toks)
    total = run = 0
    for t in response_toks:
        if t in vocab:
            run += 1
        else:
            total += run if run >= min_run else 0
            run = 0
    return total + (run if run >= min_run else 0)


def prompt_selection_for_response_generation(input_path, output_path, seed, n_out=20):
    """20 shuffled examples whose response copies 60-90 % of its tokens from the
    knowledge in long runs and covers >= 80 % of the knowledge (reference :462-530)."""
    rng = np.random.RandomState(seed)
    examples = []
    for row in _read_tsv(input_path):
        topic, turns, knowledge, response = row[0], row[1].split(" [SEP] ")[-3:], row[2], row[3]
        if knowledge == NO_KNOWLEDGE:
            continue
        k_toks, r_toks = word_tokenize(knowledge), word_tokenize(response)
        n = _overlap_tokens(k_toks, r_toks)
        if n > len(r_toks) * 0.9 or n < len(r_toks) * 0.6 or n < len(k_toks) * 0.8:
            continue
        examples.append("Topic: " + topic + ". " + "User says: " + " ".join(word_tokenize(turns[-1]))
                        + " " + "We know that: " + " ".join(k_toks) + " "
                        + "System replies: " + " ".join(r_toks))
    rng.shuffle(examples)
    with open(output_path, "w") as f:
        for e in examples[:n_out]:
            f.write(e + "\n")
    return examples[:n_out]


def prepare_input_for_response_generation(test_file, knwl_gen_file, processed_file):
    """Replace the golden knowledge column by the stage-1 generations."""
    with open(knwl_gen_file) as f:
        knowledge = [line.strip().replace("<|endoftext|>", "") for line in f]
    with open(processed_file, "w") as fw:
        for i, row in enumerate(_read_tsv(test_file)):
            fw.write("\t".join((row[0], row[1], knowledge[i], row[3])) + "\n")


def get_args(argv=None):
    p = argparse.ArgumentParser(description="MSDP preprocessing")
    p.add_argument("--func", type=str, required=True,
                   choices=["process_wow_dataset", "process_woi_dataset", "get_knwl_gen_prompts",
                            "get_resp_gen_prompts", "prepare_input"])
    for name in ("raw_file", "processed_file", "knwl_ref_file", "resp_ref_file", "knwl_gen_file",
                 "test_file", "train_file", "model_file", "data_type"):
        p.add_argument("--" + name, type=str, default=None)
    p.add_argument("--seed", type=int, default=1234)
    return p.parse_args(argv)


def main(argv=None):
    a = get_args(argv)
    if a.func == "process_wow_dataset":
        process_wow_dataset(a.raw_file, a.processed_file, a.knwl_ref_file, a.resp_ref_file)
    elif a.func == "process_woi_dataset":
        process_woi_dataset(a.raw_file, a.processed_file, a.knwl_ref_file, a.resp_ref_file)
    elif a.func == "get_knwl_gen_prompts":
        prompt_selection_for_knowledge_generation(a.test_file, a.train_file, a.model_file,
                                                  a.processed_file, a.data_type)
    elif a.func == "get_resp_gen_prompts":
        prompt_selection_for_response_generation(a.train_file, a.processed_file, a.seed)
    else:
        prepare_input_for_response_generation(a.test_file, a.knwl_gen_file, a.processed_file)


if __name__ == "__main__":
    main()

"""MSDP-PROMPT: few-shot prompting of a pretrained LM for knowledge / response
generation (reference ``tasks/msdp/prompt.py``).

Stage 1 (``--prompt_type knowledge``): per test sample, the prompt is the
sample-specific list of ``( last turn ) topic => knowledge`` examples selected
by ``preprocessing.py get_knwl_gen_prompts`` (a JSONL of
``{"<topic> <last turn>": [examples...]}``), followed by
``( <last turn> ) <topic> =>``.
Stage 2 (``--prompt_type response``): a fixed prompt of the first
``--num_prompt_examples`` lines of the prompt file, followed by
``Topic: ... User says: ... We know that: ... System replies:``.

Generation is greedy (top-k 1), ``--out_seq_length`` new tokens, and only the
first generated line is kept (reference :270-277).  Two back ends:
``--api_prompt`` PUTs to a running text-generation server
(``--megatron_api_url``; reference :19-35) and the default runs the model
in-process over TP/PP with the KV-cached generator.  Unlike the reference,
which decodes one sample per call, in-process generation batches
``--micro_batch_size`` samples per call (left context lengths may differ: the
generator handles ragged prompts), which keeps the MFMA GEMMs fed.
"""
import json

import torch

from epfl_megatron_amd import get_args, print_rank_0
from epfl_megatron_amd.parallel import state

from .metrics import word_tokenize


def _join(examples):
    return "".join(e.strip() + " \n" for e in examples)


def read_prompts(prompt_path, prompt_type, n_example):
    """knowledge -> {key: prompt text} (first occurrence of a key wins);
    response -> one prompt text from the first ``n_example`` lines."""
    if prompt_type == "knowledge":
        prompts = {}
        with open(prompt_path) as f:
            for line in f:
                if not line.strip():
                    continue
                entry = json.loads(line)
                key = next(iter(entry))
                prompts.setdefault(key, _join(entry[key]))
        return prompts
    with open(prompt_path) as f:
        return _join(f.readlines()[:n_example])


def build_input(sample_line, prompt_type, prompts):
    """Prompt text for one ``topic \\t context \\t knowledge \\t response`` line."""
    splits = sample_line.strip().split("\t")
    topic = splits[0]
    last_turn = splits[1].split(" [SEP] ")[-1]
    if prompt_type == "knowledge":
        return prompts[topic + " " + last_turn] + "( " + last_turn + " ) " + topic + " =>"
    knowledge = " ".join(word_tokenize(splits[2])).strip()
    last_turn = " ".join(word_tokenize(last_turn)).strip()
    return (prompts + "Topic: " + topic + ". " + "User says: " + last_turn + " "
            + "We know that: " + knowledge + " " + "System replies:")


def postprocess(prompt, full_text):
    """First line of the continuation (prompt text stripped off)."""
    return full_text[len(prompt):].split("\n")[0].strip()


def call_model_api(inputs, tokens_to_generate, url):
    import requests
    data = {"prompts": [inputs], "tokens_to_generate": tokens_to_generate, "top_k": 1}
    out = requests.put(url, headers={"Content-Type": "application/json; charset=UTF-8"},
                       data=json.dumps(data)).json()["text"][0]
    return postprocess(inputs, out)


def run_prompting(sample_lines, prompt_type, prompts, generate_batch, batch_size=1):
    """Generic loop: ``generate_batch(list_of_prompts) -> list_of_full_texts``."""
    outputs = []
    for i in range(0, len(sample_lines), batch_size):
        inputs = [build_input(s, prompt_type, prompts) for s in sample_lines[i:i + batch_size]]
        texts = generate_batch(inputs)
        outputs.extend(postprocess(p, t) for p, t in zip(inputs, texts))
        if (i // batch_size) % 100 == 0:
            print_rank_0(f"input_pos: {i + len(inputs)}")
    return outputs


def _read_samples(path):
    with open(path) as f:
        return [line for line in f if line.strip()]


def _write(path, lines):
    with open(path, "w") as f:
        for line in lines:
            f.write(line + "\n")


def generate_samples_by_calling_api():
    args = get_args()
    prompts = read_prompts(args.prompt_file, args.prompt_type, args.num_prompt_examples)
    samples = _read_samples(args.sample_input_file)
    outs = run_prompting(
        samples, args.prompt_type, prompts,
        lambda batch: [p + call_model_api(p, args.out_seq_length, args.megatron_api_url)
                       for p in batch])
    _write(args.sample_output_file, outs)


def model_provider(pre_process=True, post_process=True):
    import finetune
    model = finetune.model_provider(pre_process, post_process)
    model.parallel_output = True
    return model


def generate_samples_by_prompting_input_from_file(model):
    """Every rank walks the same samples (the generator broadcasts tokens across
    TP/PP); only the first-stage TP-rank-0 process writes the output file."""
    from epfl_megatron_amd.inference import generate_and_post_process
    args = get_args()
    assert args.sample_input_file is not None, "sample input file is not provided."
    assert args.prompt_type in ("knowledge", "response"), "Please input a correct prompt type!"
    out_path = args.sample_output_file or args.sample_input_file + ".out"
    prompts = read_prompts(args.prompt_file, args.prompt_type, args.num_prompt_examples)
    samples = _read_samples(args.sample_input_file)

    def gen(batch):
        out = generate_and_post_process(model, prompts=batch,
                                        tokens_to_generate=args.out_seq_length,
                                        top_k_sampling=1)
        return out[0] if out is not None else [""] * len(batch)

    model.eval()
    with torch.no_grad():
        outs = run_prompting(samples, args.prompt_type, prompts, gen,
                             batch_size=max(1, args.micro_batch_size))
    if state.is_pipeline_first_stage() and state.get_tensor_model_parallel_rank() == 0:
        _write(out_path, outs)
    return outs


def main():
    args = get_args()
    if args.api_prompt:
        return generate_samples_by_calling_api()
    if args.num_layers_per_virtual_pipeline_stage is not None:
        raise SystemExit("Interleaved pipeline schedule is not supported for text generation.")
    from epfl_megatron_amd.checkpointing import load_checkpoint
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.training import get_model
    model = get_model(model_provider, ModelType.encoder_or_decoder, wrap_with_ddp=False)
    if args.load is not None:
        load_checkpoint(model, None, None)
    assert len(model) == 1
    return generate_samples_by_prompting_input_from_file(model[0])

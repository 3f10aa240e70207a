"""Public inference API (reference ``megatron/text_generation/api.py``).

Request parameters given on rank 0 are broadcast to every rank as one float
vector, prompts are tokenised on rank 0 and broadcast, then all ranks run the
same generation loop.
"""
import torch

from ..parallel import comm, state
from .communication import broadcast_float_list, device
from .generation import (beam_search_and_return_on_first_stage,
                         generate_tokens_probs_and_return_on_first_stage,
                         score_and_return_on_first_stage)
from .tokenization import detokenize_generations, tokenize_prompts


def generate_and_post_process(model, prompts=None, tokens_to_generate=0,
                              return_output_log_probs=False, top_k_sampling=0,
                              top_p_sampling=0.0, top_p_decay=0.0, top_p_bound=0.0,
                              temperature=1.0, add_BOS=False,
                              use_eod_token_for_early_termination=True, stop_on_double_eol=False,
                              stop_on_eol=False, prevent_newline_after_colon=False,
                              random_seed=-1):
    """-> (texts, per-token segments, log-probs, tokens) on the first stage, else None."""
    tokens, lengths, logp = generate(
        model, prompts=prompts, tokens_to_generate=tokens_to_generate,
        return_output_log_probs=return_output_log_probs, top_k_sampling=top_k_sampling,
        top_p_sampling=top_p_sampling, top_p_decay=top_p_decay, top_p_bound=top_p_bound,
        temperature=temperature, add_BOS=add_BOS,
        use_eod_token_for_early_termination=use_eod_token_for_early_termination,
        stop_on_double_eol=stop_on_double_eol, stop_on_eol=stop_on_eol,
        prevent_newline_after_colon=prevent_newline_after_colon, random_seed=random_seed)
    if not state.is_pipeline_first_stage():
        return None
    tokens, texts, segments = detokenize_generations(tokens, lengths, True)
    if return_output_log_probs:
        logp = logp.cpu().numpy().tolist()
        logp = [lp[:len(seg) - 1] for lp, seg in zip(logp, segments)]
    return texts, segments, logp, tokens


def generate(model, prompts=None, tokens_to_generate=0, return_output_log_probs=False,
             top_k_sampling=0, top_p_sampling=0.0, top_p_decay=0.0, top_p_bound=0.0,
             temperature=1.0, add_BOS=False, use_eod_token_for_early_termination=True,
             stop_on_double_eol=False, stop_on_eol=False, prevent_newline_after_colon=False,
             random_seed=-1):
    """-> (tokens [b, :], lengths incl. prompt [b], log-probs or None)."""
    vals = broadcast_float_list(13, float_list=[
        tokens_to_generate, return_output_log_probs, top_k_sampling, top_p_sampling,
        top_p_decay, top_p_bound, temperature, add_BOS, use_eod_token_for_early_termination,
        stop_on_double_eol, stop_on_eol, prevent_newline_after_colon, random_seed]).tolist()
    (tokens_to_generate, return_output_log_probs, top_k_sampling, top_p_sampling, top_p_decay,
     top_p_bound, temperature, add_BOS, use_eod, stop_on_double_eol, stop_on_eol,
     prevent_newline_after_colon, random_seed) = vals
    tokens_to_generate, top_k_sampling, random_seed = (int(tokens_to_generate),
                                                       int(top_k_sampling), int(random_seed))
    if random_seed != -1:
        torch.random.manual_seed(random_seed)
    toks, lens = tokenize_prompts(prompts=prompts, tokens_to_generate=tokens_to_generate,
                                  add_BOS=bool(add_BOS))
    if tokens_to_generate == 0:
        out = score_and_return_on_first_stage(model, toks, lens)
    else:
        out = generate_tokens_probs_and_return_on_first_stage(
            model, toks, lens, return_output_log_probs=bool(return_output_log_probs),
            top_k=top_k_sampling, top_p=top_p_sampling, top_p_decay=top_p_decay,
            top_p_bound=top_p_bound, temperature=temperature,
            use_eod_token_for_early_termination=bool(use_eod),
            stop_on_double_eol=bool(stop_on_double_eol), stop_on_eol=bool(stop_on_eol),
            prevent_newline_after_colon=bool(prevent_newline_after_colon))
    comm.check_xgmi()  # a one-shot TP collective that timed out poisoned the tokens: raise
    return out


def beam_search_and_post_process(model, prompts=None, tokens_to_generate=0, beam_size=0,
                                 add_BOS=False, stop_token=50256, num_return_gen=1,
                                 length_penalty=1, prevent_newline_after_colon=False):
    tokens, scores = beam_search(model, prompts=prompts, tokens_to_generate=tokens_to_generate,
                                 beam_size=beam_size, add_BOS=add_BOS, stop_token=stop_token,
                                 num_return_gen=num_return_gen, length_penalty=length_penalty,
                                 prevent_newline_after_colon=prevent_newline_after_colon)
    if not state.is_pipeline_first_stage():
        return None
    lengths = torch.full((tokens.size(0),), tokens.size(1), dtype=torch.int64, device=device())
    _, texts, segments = detokenize_generations(tokens, lengths, True)
    return texts, segments, scores.cpu().numpy().tolist()


def beam_search(model, prompts=None, tokens_to_generate=0, beam_size=0, add_BOS=False,
                stop_token=50256, num_return_gen=1, length_penalty=1,
                prevent_newline_after_colon=False):
    vals = broadcast_float_list(7, float_list=[
        tokens_to_generate, beam_size, add_BOS, stop_token, num_return_gen, length_penalty,
        prevent_newline_after_colon]).tolist()
    tokens_to_generate, beam_size, add_BOS, stop_token, num_return_gen = (
        int(vals[0]), int(vals[1]), bool(vals[2]), int(vals[3]), int(vals[4]))
    length_penalty, prevent_newline_after_colon = vals[5], bool(vals[6])
    toks, lens = tokenize_prompts(prompts=prompts, tokens_to_generate=tokens_to_generate,
                                  add_BOS=add_BOS)
    out = beam_search_and_return_on_first_stage(
        model, toks, lens, beam_size, stop_token=stop_token, num_return_gen=num_return_gen,
        length_penalty=length_penalty, prevent_newline_after_colon=prevent_newline_after_colon)
    comm.check_xgmi()
    return out

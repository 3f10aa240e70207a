"""Scoring, sampling generation and beam search over a KV-cached model
(reference ``megatron/text_generation/generation.py``).

All loops follow the reference's contract: inputs are available on every
rank, logits only on the last pipeline stage, results are returned on the
first stage, and each new token is copied from the last to the first stage so
the next step's embedding lookup sees it.  The first step pre-fills the cache
with the shortest prompt; later steps feed one token.
"""
import torch
import torch.nn.functional as F

from .. import global_vars
from ..parallel import state
from ..utils.misc import get_ltor_masks_and_position_ids
from .beam_utils import BeamHypotheses
from .communication import (broadcast_from_last_pipeline_stage,
                            broadcast_from_last_to_first_pipeline_stage,
                            copy_from_last_to_first_pipeline_stage, device)
from .forward_step import ForwardStep
from .sampling import sample


def _check_budget(args, seq_len, batch):
    if seq_len > args.max_position_embeddings:
        raise ValueError("Length of prompt + tokens_to_generate longer than allowed")
    if seq_len * batch > args.max_tokens_to_oom:
        raise ValueError(f"Too many tokens.  {seq_len * batch} is greater than "
                         f"{args.max_tokens_to_oom}")


def _build_attention_mask_and_position_ids(tokens):
    mask, _, pos = get_ltor_masks_and_position_ids(tokens, None, False, False, False)
    return mask, pos


def _single_token_id(tokenizer, text):
    try:
        ids = tokenizer.tokenize(text)
    except Exception:
        return None
    return ids[-1] if ids else None


def score_and_return_on_first_stage(model, tokens, lengths):
    """Log-probabilities of every prompt token given its prefix: ``[b, s-1]``."""
    args = global_vars.get_args()
    b = tokens.size(0)
    s = int(lengths.max().item())
    if s != tokens.size(1):
        raise AssertionError("scoring expects unpadded prompts (tokens_to_generate == 0)")
    _check_budget(args, s, b)
    step = ForwardStep(model, b, s)
    out = None
    with torch.no_grad():
        mask, pos = _build_attention_mask_and_position_ids(tokens)
        logits = step(tokens, pos, mask)
        if state.is_pipeline_last_stage():
            logp = F.log_softmax(logits.float(), dim=2)
            out = torch.gather(logp, 2, tokens[:, 1:].unsqueeze(2)).squeeze(2).contiguous()
    out = broadcast_from_last_to_first_pipeline_stage((b, s - 1), torch.float32, out)
    return tokens, lengths, out


def generate_tokens_probs_and_return_on_first_stage(
        model, tokens, lengths, return_output_log_probs=False, top_k=0, top_p=0.0,
        top_p_decay=0.0, top_p_bound=0.0, temperature=1.0,
        use_eod_token_for_early_termination=True, stop_on_double_eol=False, stop_on_eol=False,
        prevent_newline_after_colon=True):
    args = global_vars.get_args()
    tokenizer = global_vars.get_tokenizer()
    b = tokens.size(0)
    min_len = int(lengths.min().item())
    max_len = tokens.size(1)
    _check_budget(args, max_len, b)
    step = ForwardStep(model, b, max_len)
    termination_id = getattr(args, "eos_id", None)
    if termination_id is None:
        termination_id = tokenizer.eod
    eol = _single_token_id(tokenizer, "\n")
    double_eol = _single_token_id(tokenizer, "\n\n")
    colon = _single_token_id(tokenizer, ":") if prevent_newline_after_colon else None
    dev = device()
    last = state.is_pipeline_last_stage()
    logp_out = torch.empty((b, max_len - 1), dtype=torch.float32, device=dev) \
        if (last and return_output_log_probs) else None
    gen_lengths = torch.full((b,), max_len, dtype=torch.int64, device=dev) if last else None
    done_mask = torch.zeros(b, dtype=torch.uint8, device=dev)
    context_length = min_len
    with torch.no_grad():
        mask, pos = _build_attention_mask_and_position_ids(tokens)
        prev = 0
        for context_length in range(min_len, max_len):
            toks = tokens[:, prev:context_length]
            logits = step(toks, pos[:, prev:context_length],
                          mask[..., prev:context_length, :context_length])
            done = None
            if last:
                logits = logits.float()
                if prevent_newline_after_colon and colon is not None and eol is not None:
                    logits[toks[:, -1] == colon, -1, eol] = -1e10
                new = sample(logits[:, -1, :].contiguous(), top_k=top_k, top_p=top_p,
                             temperature=temperature, vocab_size=tokenizer.vocab_size)
                if top_p > 0.0 and top_p_decay > 0.0:
                    top_p = max(top_p * top_p_decay, top_p_bound) if top_p_bound > 0.0 \
                        else top_p * top_p_decay
                started = lengths <= context_length
                tokens[started, context_length] = new[started]
                if return_output_log_probs:
                    lp = F.log_softmax(logits, dim=2)
                    idx = tokens[:, prev + 1:context_length + 1].unsqueeze(2)
                    logp_out[:, prev:context_length] = torch.gather(lp, 2, idx).squeeze(2)
                if stop_on_double_eol or stop_on_eol:
                    hit = torch.zeros_like(started)
                    if double_eol is not None:
                        hit |= new == double_eol
                    if eol is not None:
                        if stop_on_double_eol:
                            hit |= (new == eol) & (tokens[:, context_length - 1] == eol)
                        else:
                            hit |= new == eol
                    done_tok = (hit & started).to(torch.uint8)
                else:
                    done_tok = ((new == termination_id) & started).to(torch.uint8)
                just = (done_tok & (1 - done_mask)).bool()
                gen_lengths[just] = context_length + 1
                done_mask |= done_tok
                done = torch.all(done_mask.bool()).to(torch.uint8).view(1)
            copy_from_last_to_first_pipeline_stage(b, torch.int64, tokens[:, context_length])
            prev = context_length
            done = broadcast_from_last_pipeline_stage(1, torch.uint8, done)
            if use_eod_token_for_early_termination and bool(done.item()):
                break
    tokens = tokens[:, :context_length + 1]
    if logp_out is not None:
        logp_out = logp_out[:, :context_length].contiguous()
    gen_lengths = broadcast_from_last_to_first_pipeline_stage(b, torch.int64, gen_lengths)
    if return_output_log_probs:
        logp_out = broadcast_from_last_to_first_pipeline_stage((b, context_length),
                                                               torch.float32, logp_out)
    return tokens, gen_lengths, logp_out


def beam_search_and_return_on_first_stage(model, tokens, lengths, beam_size, stop_token,
                                          num_return_gen, length_penalty,
                                          prevent_newline_after_colon=True):
    args = global_vars.get_args()
    tokenizer = global_vars.get_tokenizer()
    if tokens.size(0) != 1:
        raise AssertionError("beam search takes a single prompt")
    prompt_len = int(lengths.item())
    final_len = min(tokens.size(1), args.max_position_embeddings)
    if prompt_len >= final_len:
        raise ValueError("context length + tokens_to_generate too large")
    step = ForwardStep(model, beam_size, final_len)
    hyps = BeamHypotheses(beam_size, length_penalty)
    dev = device()
    last = state.is_pipeline_last_stage()
    done = torch.zeros(1, dtype=torch.uint8, device=dev)
    scores = torch.zeros(beam_size, 1, dtype=torch.float32, device=dev)
    eol = _single_token_id(tokenizer, "\n")
    colon = _single_token_id(tokenizer, ":") if prevent_newline_after_colon else None
    best = None
    context_length = prompt_len
    with torch.no_grad():
        tokens = tokens.repeat(beam_size, 1)
        mask, pos = _build_attention_mask_and_position_ids(tokens)
        prev = 0
        for context_length in range(prompt_len, final_len):
            toks = tokens[:, prev:context_length]
            logits = step(toks, pos[:, prev:context_length],
                          mask[..., prev:context_length, :context_length])
            if last:
                logits = logits.float()
                if prevent_newline_after_colon and colon is not None and eol is not None:
                    logits[toks[:, -1] == colon, -1, eol] = -1e10
                vocab = logits.size(2)
                cand = F.log_softmax(logits, dim=2)[:, -1, :] + scores
                flat = cand[0] if context_length == prompt_len else cand.view(-1)
                top_scores, top_idx = torch.topk(flat, 2 * beam_size)
                next_beams = []
                for rank, (idx, sc) in enumerate(zip(top_idx.tolist(), top_scores.tolist())):
                    beam_id, token_id = divmod(idx, vocab)
                    if token_id == stop_token:
                        if rank < beam_size:
                            hyps.add(tokens[beam_id].clone(), sc,
                                     context_length + 1 - prompt_len)
                    else:
                        next_beams.append((token_id, sc, beam_id))
                    if len(next_beams) == beam_size:
                        break
                if hyps.is_done(top_scores.max().item(), context_length + 1 - prompt_len):
                    done = torch.ones(1, dtype=torch.uint8, device=dev)
                best = torch.tensor([nb[2] for nb in next_beams], dtype=torch.int64, device=dev)
                tokens = tokens[best, :]
                tokens[:, context_length] = torch.tensor([nb[0] for nb in next_beams],
                                                         dtype=torch.int64, device=dev)
                scores = torch.tensor([nb[1] for nb in next_beams], dtype=torch.float32,
                                      device=dev).unsqueeze(1)
            done = broadcast_from_last_pipeline_stage(1, torch.uint8, done)
            if bool(done.item()):
                break
            copy_from_last_to_first_pipeline_stage(tokens.size(), torch.int64, tokens)
            best = broadcast_from_last_pipeline_stage(beam_size, torch.int64, best)
            step.inference_params.swap_key_value_dict(best)
            prev = context_length
        out_scores = out_tokens = None
        s_size = t_size = None
        if last:
            if not bool(done.item()):
                for i in range(beam_size):
                    hyps.add(tokens[i].clone(), scores[i].squeeze(), context_length + 1 - prompt_len)
            ranked = sorted(hyps.beams, key=lambda x: x[0], reverse=True)
            n = min(num_return_gen, len(ranked))
            out_scores = torch.tensor([float(r[0]) for r in ranked[:n]], dtype=torch.float32,
                                      device=dev)
            width = max(r[1].numel() for r in ranked[:n])
            out_tokens = torch.stack([F.pad(r[1], (0, width - r[1].numel()),
                                            value=tokenizer.eod) for r in ranked[:n]])
            s_size = torch.tensor(out_scores.shape, dtype=torch.int64, device=dev)
            t_size = torch.tensor(out_tokens.shape, dtype=torch.int64, device=dev)
        s_size = broadcast_from_last_pipeline_stage(1, torch.int64, s_size)
        t_size = broadcast_from_last_pipeline_stage(2, torch.int64, t_size)
        out_scores = broadcast_from_last_to_first_pipeline_stage(tuple(s_size.tolist()),
                                                                 torch.float32, out_scores)
        out_tokens = broadcast_from_last_to_first_pipeline_stage(tuple(t_size.tolist()),
                                                                 torch.int64, out_tokens)
    return out_tokens, out_scores

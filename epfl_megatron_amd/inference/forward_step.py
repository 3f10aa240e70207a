"""Incremental (KV-cached) forward for generation (reference
``megatron/text_generation/forward_step.py``).

``InferenceParams`` owns the per-layer KV caches (allocated lazily by each
attention layer as ``[max_seq, max_batch, nkv_per_tp, hd]`` — GQA keys stay at
``nkv`` heads, already rotated) and the running sequence / batch offsets.
``ForwardStep`` runs one model call per generation step across pipeline
stages; when ``batch x new_tokens`` exceeds
``--inference_batch_times_seqlen_threshold`` the batch is split into
micro-batches that stream through the pipeline (prefill of long prompts).
"""
from collections.abc import Iterable

import torch

from .. import global_vars
from ..parallel import state
from .communication import device, recv_from_prev_pipeline_rank_, send_to_next_pipeline_rank


class InferenceParams:

    def __init__(self, max_batch_size, max_sequence_len):
        self.max_sequence_len = max_sequence_len
        self.max_batch_size = max_batch_size
        self.sequence_len_offset = 0
        self.batch_size_offset = 0
        self.key_value_memory_dict = {}
        # hipGraph decode (inference/hip_graph.py): the cache slot of the new
        # token (int64 [1]) and the valid key count (int32 [1]) on the device
        self.device_offset = None
        self.device_kv_len = None

    def swap_key_value_dict(self, batch_idx):
        """Reorder the cached batch rows (beam search keeps the best beams)."""
        if not self.key_value_memory_dict:
            raise ValueError("should not swap when dict in empty")
        for layer, (k, v) in self.key_value_memory_dict.items():
            if len(batch_idx) != k.shape[1]:
                raise AssertionError("batch size mismatch while reordering the KV cache")
            # in place: a captured hipGraph (inference/hip_graph.py) holds
            # these cache addresses
            k.copy_(k[:, batch_idx])
            v.copy_(v[:, batch_idx])


class ForwardStep:

    def __init__(self, model, max_batch_size, max_sequence_len):
        if isinstance(model, Iterable):
            raise AssertionError("interleaving schedule is not supported for inference")
        model.eval()
        self.model = model
        self.inference_params = InferenceParams(max_batch_size, max_sequence_len)
        args = global_vars.get_args()
        self.pipelined = args.pipeline_model_parallel_size > 1
        self.threshold = args.inference_batch_times_seqlen_threshold
        self.graphed = None
        if getattr(args, "inference_hip_graph", False):
            # a hipGraph per pipeline stage on the GPU; on the CPU the same
            # static-buffer step runs eagerly
            from .hip_graph import GraphedDecodeForward
            self.graphed = GraphedDecodeForward(model, self.inference_params, max_batch_size)

    def __call__(self, tokens, position_ids, attention_mask):
        if self.graphed is not None and tokens.size(1) == 1 and \
                tokens.size(0) == self.inference_params.max_batch_size:
            out = self.graphed(tokens, position_ids)
            self.inference_params.sequence_len_offset += 1
            return out
        if self.pipelined and tokens.size(0) * tokens.size(1) >= self.threshold:
            mbs = max(1, self.threshold // tokens.size(1))
            return _with_pipelining_forward_step(self.model, tokens, position_ids,
                                                 attention_mask, self.inference_params, mbs)
        return _no_pipelining_forward_step(self.model, tokens, position_ids, attention_mask,
                                           self.inference_params)


def _recv_dtype(args):
    return torch.float if args.fp32_residual_connection else args.params_dtype


def _allocate_recv_buffer(batch_size, sequence_length):
    if state.is_pipeline_first_stage():
        return None
    args = global_vars.get_args()
    return torch.empty((sequence_length, batch_size, args.hidden_size), dtype=_recv_dtype(args),
                       device=device())


def _forward_step_helper(model, tokens, position_ids, attention_mask, inference_params,
                         recv_buffer=None):
    if recv_buffer is None:
        recv_buffer = _allocate_recv_buffer(tokens.size(0), tokens.size(1))
    recv_from_prev_pipeline_rank_(recv_buffer)
    model.set_input_tensor(recv_buffer)
    out = model(tokens, position_ids, attention_mask, inference_params=inference_params)
    send_to_next_pipeline_rank(out)
    return out


def _no_pipelining_forward_step(model, tokens, position_ids, attention_mask, inference_params,
                                recv_buffer=None):
    out = _forward_step_helper(model, tokens, position_ids, attention_mask, inference_params,
                               recv_buffer)
    inference_params.sequence_len_offset += tokens.size(1)
    return out if state.is_pipeline_last_stage() else None


def _with_pipelining_forward_step(model, tokens, position_ids, attention_mask, inference_params,
                                  micro_batch_size):
    b, s = tokens.shape
    logits = None
    if state.is_pipeline_last_stage():
        args = global_vars.get_args()
        logits = torch.empty((b, s, args.padded_vocab_size), dtype=torch.float32,
                             device=device())
    recv = _allocate_recv_buffer(micro_batch_size, s)
    for start in range(0, b, micro_batch_size):
        end = min(start + micro_batch_size, b)
        out = _forward_step_helper(model, tokens[start:end], position_ids[start:end],
                                   attention_mask, inference_params,
                                   recv if end - start == micro_batch_size else None)
        inference_params.batch_size_offset += end - start
        if logits is not None:
            logits[start:end] = out
    inference_params.sequence_len_offset += s
    inference_params.batch_size_offset = 0
    return logits

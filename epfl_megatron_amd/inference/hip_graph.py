"""hipGraph-captured decode step for KV-cached generation on MI355X.

One token-by-token decode step of Llama-2-7B issues ~450 small launches
(per layer: fused-QKV skinny GEMM, RoPE, two cache writes, split-key decode
attention + combine, dense, residual-norm, fc1, SwiGLU, fc2, ...).  Eagerly
the host issuing them sets the pace; captured ONCE into a HIP graph
(``torch.cuda.CUDAGraph`` is a hipGraph on ROCm) and replayed there is no
Python and no per-kernel launch cost: 4.19 ms/step at batch 1 vs 4.8-5.7
eager, 5.6 vs 7.0-8.2 at batch 32 (``profiles/r2f_serve_graph.txt``).

What makes the step capturable: nothing in it depends on the step on the host.
  * the token's cache slot and the number of valid keys are device tensors
    (``InferenceParams.device_offset`` / ``device_kv_len``): the K/V write is
    an ``index_copy_`` and the decode attention reads the key count on the
    device (``csrc/flash_decode.hip``, grid sized for the whole cache, chunks
    past the length exit early);
  * RoPE takes the absolute position ids (a static device tensor);
  * ``GraphedGreedyDecoder``: greedy selection (argmax), the position /
    slot / length increments and the write into the generated-token history
    are part of the graph (no host work per token at all);
  * ``GraphedDecodeForward`` (``--inference_hip_graph``, used by
    ``ForwardStep`` and so by the text-generation API and server): only the
    forward is replayed, sampling and stop conditions stay eager.

Tensor parallelism: every TP rank captures its own graph of the same step;
the row-parallel all-reduces (two [b, h] sums per layer in the fused decode
layer, ``models/transformer.py``) and the vocab all-gather of the logits are
RCCL collectives recorded into the graph (RCCL kernels are capturable; the
communicator is created by the eager warm-up forward, before capture, and the
collective layer records no timing events while capturing).  All TP ranks run
the generation loop in lockstep, as the reference's TP generation does
(``megatron/text_generation/generation.py:179-264``), so every replay issues
the same collective sequence on every rank.

Pipeline parallelism (``GraphedDecodeForward``): every stage captures its own
layers; the stage boundaries stay eager p2p around the replay (the hidden
state is received into a static buffer the graph reads, the static output is
sent after the replay), as the reference's PP forward step does
(``megatron/text_generation/forward_step.py:153-204``).  The launch-bound part
(tens of small kernels per layer) is in the graph; one send / recv per stage
per token is not.  ``GraphedGreedyDecoder`` (argmax and the token feedback in
the graph) needs the whole model on the rank: PP = 1.  Without a GPU the
same static-buffer step runs eagerly (the CPU / gloo tests drive the PP
plumbing through it).

The reference decodes eagerly (``megatron/text_generation/generation.py``
drives ``forward_step.py`` once per token); this is an MI355X-side addition.
"""
import torch

from ..parallel import state


def _check_supported():
    if state.model_parallel_is_initialized() and state.get_pipeline_model_parallel_world_size() > 1:
        raise NotImplementedError("the graphed greedy loop needs the whole model (PP = 1); "
                                  "GraphedDecodeForward runs per pipeline stage")
    if not torch.cuda.is_available():
        raise RuntimeError("hipGraph decode needs a GPU")


def graph_decode_supported():
    """GraphedDecodeForward captures on a GPU at any TP / PP size."""
    return torch.cuda.is_available()


def _pp_stage():
    """(first stage, last stage) of this rank (a single stage without PP)."""
    if not state.model_parallel_is_initialized():
        return True, True
    return state.is_pipeline_first_stage(), state.is_pipeline_last_stage()


class GraphedDecodeForward:
    """The single-token model forward of ``ForwardStep`` (``--inference_hip_graph``):
    inputs are copied into static tensors, the cache slot / key count are
    set from ``inference_params.sequence_len_offset`` on the device, and the
    captured forward is replayed.  Sampling, stop conditions and log-probs
    stay in the (eager) generation loop.  Returns the static logits buffer,
    valid until the next call."""

    def __init__(self, model, inference_params, batch, capture=None):
        self.model = model
        self.ip = inference_params
        self.capture = torch.cuda.is_available() if capture is None else capture
        dev = torch.device("cuda", torch.cuda.current_device()) if self.capture else \
            torch.device("cpu")
        self.tokens = torch.zeros(batch, 1, dtype=torch.long, device=dev)
        self.pos = torch.zeros(batch, 1, dtype=torch.long, device=dev)
        self.ip.device_offset = torch.zeros(1, dtype=torch.long, device=dev)
        self.ip.device_kv_len = torch.zeros(1, dtype=torch.int32, device=dev)
        self.first, self.last = _pp_stage()
        self.recv = None
        if not self.first:  # static input of this stage's graph: the previous stage's output
            from .forward_step import _allocate_recv_buffer
            self.recv = _allocate_recv_buffer(batch, 1)
        self.graph = None
        self.out = None

    def _forward(self):
        if self.recv is not None:
            self.model.set_input_tensor(self.recv)
        return self.model(self.tokens, self.pos, None, inference_params=self.ip)

    def __call__(self, tokens, position_ids):
        """One decode step of this stage: the logits on the last stage, None on
        the others (their output went to the next stage)."""
        from .communication import recv_from_prev_pipeline_rank_, send_to_next_pipeline_rank
        ip = self.ip
        with torch.no_grad():
            self.tokens.copy_(tokens)
            self.pos.copy_(position_ids)
            ip.device_offset.fill_(ip.sequence_len_offset)
            ip.device_kv_len.fill_(ip.sequence_len_offset + 1)
            if self.recv is not None:
                recv_from_prev_pipeline_rank_(self.recv)
            if not self.capture:
                self.out = self._forward()
            elif self.graph is None:
                cur = torch.cuda.current_stream()
                side = torch.cuda.Stream()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    self._forward()  # warm-up; rewrites the same cache slot
                cur.wait_stream(side)
                self.graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph):
                    self.out = self._forward()
            if self.graph is not None:
                self.graph.replay()
            if not self.last:
                send_to_next_pipeline_rank(self.out)
        return self.out if self.last else None


class GraphedGreedyDecoder:
    """Greedy decode of ``batch`` sequences whose prompts were prefilled into
    ``inference_params`` (eagerly, e.g. one ``model(prompt, ...)`` call).

    Usage::

        dec = GraphedGreedyDecoder(model, ip, batch, max_new_tokens)
        dec.start(next_tokens, position)   # first new token, its position
        for _ in range(n):
            dec.step()                     # one replay = one generated token
        tokens = dec.history[:, :n]        # [batch, n] (device)
    """

    def __init__(self, model, inference_params, batch, max_new_tokens):
        _check_supported()
        self.model = model
        self.ip = inference_params
        self.batch = batch
        self.max_new = max_new_tokens
        dev = torch.device("cuda", torch.cuda.current_device())
        self.tokens = torch.zeros(batch, 1, dtype=torch.long, device=dev)
        self.pos = torch.zeros(batch, 1, dtype=torch.long, device=dev)
        self.step_idx = torch.zeros(1, dtype=torch.long, device=dev)
        self.history = torch.zeros(batch, max_new_tokens + 1, dtype=torch.long, device=dev)
        self.ip.device_offset = torch.zeros(1, dtype=torch.long, device=dev)
        self.ip.device_kv_len = torch.zeros(1, dtype=torch.int32, device=dev)
        self.tail_counter = torch.zeros(1, dtype=torch.int32, device=dev)
        self.graph = None
        self.logits = None
        self.steps_done = 0

    def _forward(self):
        return self.model(self.tokens, self.pos, None, inference_params=self.ip)

    def _body(self):
        logits = self._forward()
        last = logits[:, -1]
        if self._fused_tail(last):
            # argmax, token / history writes and the four increments in one
            # launch (csrc/decode_tail.hip; seven launches otherwise)
            from ..ops._ext import ext
            ext().greedy_tail(last, self.tokens.view(-1), self.history, self.step_idx,
                              self.pos.view(-1), self.ip.device_offset, self.ip.device_kv_len,
                              self.tail_counter)
            return logits
        nxt = last.argmax(-1, keepdim=True)
        self.history.index_copy_(1, self.step_idx, nxt)
        self.tokens.copy_(nxt)
        self.pos.add_(1)
        self.step_idx.add_(1)
        self.ip.device_offset.add_(1)
        self.ip.device_kv_len.add_(1)
        return logits

    def _fused_tail(self, last):
        from ..ops._ext import use_native
        return (use_native(last) and last.dim() == 2 and last.stride(1) == 1
                and last.dtype in (torch.bfloat16, torch.float16, torch.float32)
                and last.data_ptr() % 16 == 0 and (last.stride(0) * last.element_size()) % 16 == 0)

    def start(self, next_tokens, position):
        """Set the first token to feed (``[batch, 1]``) at absolute ``position``
        (= the number of tokens already cached) and capture the graph on the
        first call."""
        if position + self.max_new > self.ip.max_sequence_len:
            raise ValueError("KV cache too short for max_new_tokens")
        with torch.no_grad():
            self.tokens.copy_(next_tokens.view(self.batch, 1))
            self.pos.fill_(position)
            self.step_idx.zero_()
            self.ip.device_offset.fill_(position)
            self.ip.device_kv_len.fill_(position + 1)
            if self.graph is None:
                self._capture()
        self.base = position
        self.steps_done = 0

    def _capture(self):
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            # warm-up at the current state: writes the cache slot the first
            # replay writes again (idempotent), initialises lazy state
            self._forward()
        cur.wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.logits = self._body()

    def step(self):
        if self.steps_done >= self.max_new:
            raise RuntimeError("max_new_tokens reached")
        self.graph.replay()
        self.steps_done += 1
        self.ip.sequence_len_offset = self.base + self.steps_done
        return self.tokens

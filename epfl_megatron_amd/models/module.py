"""Base module, tied-embedding sync across pipeline stages, half-precision wrapper.

Reference ``megatron/model/module.py``.  Behaviour preserved: with tied
embeddings and PP > 1 the last stage owns a zero-initialised copy of the word
embedding (``word_embeddings_for_head``) which is summed with the first
stage's copy over the embedding group once at init (and its grads are summed
every step).
"""
import torch
import torch.distributed as dist
from torch.nn.parameter import Parameter

from ..parallel import state
from ..parallel.tensor import VocabParallelEmbedding

_FLOAT_TYPES = (torch.float32,)
_HALF_TYPES = (torch.float16,)
_BF16_TYPES = (torch.bfloat16,)


def param_is_not_shared(param):
    return not getattr(param, "shared", False)


class MegatronModule(torch.nn.Module):
    def __init__(self, share_word_embeddings=True):
        super().__init__()
        self.share_word_embeddings = share_word_embeddings

    def state_dict_for_save_checkpoint(self, prefix="", keep_vars=False):
        return self.state_dict(prefix=prefix, keep_vars=keep_vars)

    def word_embeddings_weight(self):
        w = self._word_embeddings_weight()
        wait = getattr(w, "_param_sync_wait", None)
        if wait is not None:  # dist-opt: this param's all-gather may still be in flight
            wait()
        return w

    def _word_embeddings_weight(self):
        lm = self.language_model
        if self.pre_process:
            return lm.embedding.word_embeddings.weight if lm.tie_embed_logits else lm.lm_head
        if not lm.tie_embed_logits:
            return lm.lm_head
        if not self.share_word_embeddings:
            raise Exception("word_embeddings_weight() called for last stage, but "
                            "share_word_embeddings is false")
        return self.word_embeddings.weight

    def initialize_word_embeddings(self, init_method_normal, args):
        if not self.share_word_embeddings:
            raise Exception("initialize_word_embeddings() was called but share_word_embeddings "
                            "is false")
        if args.pipeline_model_parallel_size == 1:
            return
        if state.is_pipeline_last_stage() and not self.pre_process:
            self._word_embeddings_for_head_key = "word_embeddings_for_head"
            self.word_embeddings = VocabParallelEmbedding(
                args.padded_vocab_size, args.hidden_size,
                init_method=init_method_normal(args.init_method_std),
                params_dtype=args.params_dtype,
                use_cpu_initialization=args.use_cpu_initialization,
                perform_initialization=args.perform_initialization)
            with torch.no_grad():
                self.word_embeddings.weight.fill_(0)
            self.word_embeddings.weight.shared = True
        if not state.is_pipeline_first_stage(ignore_virtual=True) and self.pre_process:
            # decoder stage of a split encoder/decoder pipeline: its embeddings
            # are replicas of the first stage's (summed over the embedding /
            # position-embedding groups).  Marked shared so the grad norm counts
            # them once (the reference counts them twice).
            self.language_model.embedding.zero_parameters()
            for prm in self.language_model.embedding.parameters():
                prm.shared = True
        if not dist.is_initialized():
            return
        from ..parallel import comm  # noqa: PLC0415 (accounted, race-checked)
        if state.is_rank_in_embedding_group():
            comm.all_reduce(self.word_embeddings_weight().data, group=state.get_embedding_group())
        if state.is_rank_in_position_embedding_group() and \
                args.pipeline_model_parallel_split_rank is not None:
            pe = self.language_model.embedding.position_embeddings
            comm.all_reduce(pe.weight.data, group=state.get_position_embedding_group())


def _convert(val, fn):
    if isinstance(val, (tuple, list)):
        out = [_convert(v, fn) for v in val]
        return tuple(out) if isinstance(val, tuple) else out
    return fn(val)


def fp32_to_float16(val, float16_convertor):
    def conv(v):
        t = v.data if isinstance(v, Parameter) else v
        if isinstance(t, torch.Tensor) and t.dtype in _FLOAT_TYPES:
            return float16_convertor(v)
        return v
    return _convert(val, conv)


def float16_to_fp32(val):
    def conv(v):
        t = v.data if isinstance(v, Parameter) else v
        if isinstance(t, torch.Tensor) and t.dtype in (_BF16_TYPES + _HALF_TYPES):
            return v.float()
        return v
    return _convert(val, conv)


class Float16Module(MegatronModule):
    """Cast the wrapped module to fp16/bf16; cast float inputs on the first
    stage and outputs back to fp32 on the last stage."""

    def __init__(self, module, args):
        super().__init__()
        if args.fp16:
            self.add_module("module", module.half())
            self.float16_convertor = lambda v: v.half()
        elif args.bf16:
            self.add_module("module", module.bfloat16())
            self.float16_convertor = lambda v: v.bfloat16()
        else:
            raise Exception("should not be here")

    def set_input_tensor(self, input_tensor):
        return self.module.set_input_tensor(input_tensor)

    def forward(self, *inputs, **kwargs):
        if state.is_pipeline_first_stage():
            inputs = fp32_to_float16(inputs, self.float16_convertor)
        outputs = self.module(*inputs, **kwargs)
        if state.is_pipeline_last_stage():
            outputs = float16_to_fp32(outputs)
        return outputs

    def state_dict(self, prefix="", keep_vars=False, **kw):
        return self.module.state_dict(prefix=prefix, keep_vars=keep_vars)

    def state_dict_for_save_checkpoint(self, prefix="", keep_vars=False):
        return self.module.state_dict_for_save_checkpoint(prefix=prefix, keep_vars=keep_vars)

    def load_state_dict(self, state_dict, strict=True):
        self.module.load_state_dict(state_dict, strict=strict)

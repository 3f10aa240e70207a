"""Llama-1/2 (reference ``megatron/model/llama_model.py``): GPTModel + flag checks."""
import warnings

from .. import global_vars
from .enums import PositionEmbeddingType
from .gpt_model import GPTModel

# (predicate on args, message) — all must hold.
_REQUIRED = [
    (lambda a: a.position_embedding_type == PositionEmbeddingType.rotary,
     "Llama uses rotary embedding"),
    (lambda a: not a.use_post_ln, "Llama does not use post_ln"),
    (lambda a: a.glu_activation == "swiglu", "Llama works with swiglu activation"),
    (lambda a: not a.use_bias, "Llama does not use bias"),
    (lambda a: not a.parallel_attn, "Llama does not use parallel_attn"),
    (lambda a: a.use_rms_norm, "Llama uses rms_norm"),
    (lambda a: not a.tie_embed_logits, "Llama unties embedding and lm_head weights"),
]
_ADVISED = [
    (lambda a: not a.bias_gelu_fusion, "Llama is not intended to use bias_gelu_fusion"),
    (lambda a: not a.bias_dropout_fusion, "Llama is not intended to use bias_dropout_fusion"),
    (lambda a: a.hidden_dropout == 0.0 or a.lima_dropout, "Llama is not intended to use dropout"),
    (lambda a: a.attention_dropout == 0.0, "Llama is not intended to use dropout"),
]


def check_rules(args, required, advised):
    for pred, msg in required:
        if not pred(args):
            raise AssertionError(msg)
    for pred, msg in advised:
        if not pred(args):
            warnings.warn(msg)


class LlamaModel(GPTModel):
    def __init__(self, num_tokentypes=0, parallel_output=True, pre_process=True,
                 post_process=True, model_type=None, version=2):
        if version not in (1, 2):
            raise AssertionError(f"Unknown llama version {version}")
        check_rules(global_vars.get_args(), _REQUIRED, _ADVISED)
        super().__init__(num_tokentypes=num_tokentypes, parallel_output=parallel_output,
                         pre_process=pre_process, post_process=post_process,
                         model_type=model_type)

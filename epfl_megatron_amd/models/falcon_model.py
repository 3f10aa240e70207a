"""Falcon (reference ``megatron/model/falcon_model.py``): parallel attention/MLP,
MQA/GQA, GeLU, LayerNorm, tied embeddings."""
from .. import global_vars
from .enums import PositionEmbeddingType
from .gpt_model import GPTModel
from .llama_model import check_rules

_REQUIRED = [
    (lambda a: a.position_embedding_type == PositionEmbeddingType.rotary,
     "Falcon uses rotary embedding"),
    (lambda a: isinstance(a.num_attention_heads_kv, int),
     "Falcon needs a not None num_attention_heads_kv parameter"),
    (lambda a: not a.use_post_ln, "FalconModel requires pre-normalization, not use_post_ln"),
    (lambda a: a.glu_activation is None,
     "FalconModel requires gelu activation (set glu_activation=None)"),
    (lambda a: not a.use_bias, "Falcon does not use bias"),
    (lambda a: a.parallel_attn, "Falcon uses parallel_attn"),
]
_ADVISED = [
    (lambda a: a.parallel_layernorm, "Falcon uses parallel_layernorm, or are you running falcon-7b?"),
    (lambda a: a.use_flash_attn, "Falcon should use flash attn"),
    (lambda a: not a.bias_gelu_fusion, "Falcon should not use bias_gelu_fusion"),
    (lambda a: not a.bias_dropout_fusion, "Falcon should not use bias_dropout_fusion"),
    (lambda a: a.hidden_dropout == 0.0 or a.lima_dropout, "Falcon should not use dropout"),
]


class FalconModel(GPTModel):
    def __init__(self, num_tokentypes=0, parallel_output=True, pre_process=True,
                 post_process=True, model_type=None):
        check_rules(global_vars.get_args(), _REQUIRED, _ADVISED)
        super().__init__(num_tokentypes=num_tokentypes, parallel_output=parallel_output,
                         pre_process=pre_process, post_process=post_process,
                         model_type=model_type)

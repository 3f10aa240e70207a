"""BERT encoder with masked-LM and sentence-order heads
(reference ``megatron/model/bert_model.py``; legacy family).

State-dict keys match the reference: ``language_model``, ``lm_head``
(``bias``, ``dense``, ``layernorm``) and ``binary_head``.
"""
import torch

from .. import global_vars
from ..ops.cross_entropy import vocab_parallel_cross_entropy
from ..ops.norms import MixedFusedLayerNorm
from ..parallel import tensor as tp
from .enums import AttnMaskType
from .language_model import get_language_model, parallel_lm_logits
from .module import MegatronModule
from .utils import erf_gelu, get_linear_layer, init_method_normal, scaled_init_method_normal


def bert_extended_attention_mask(attention_mask):
    """``[b, s]`` 1 = token, 0 = pad -> bool ``[b, 1, s, s]``, True = masked out."""
    m = attention_mask.unsqueeze(1) * attention_mask.unsqueeze(2)
    return m.unsqueeze(1) < 0.5


def bert_position_ids(token_ids):
    s = token_ids.size(1)
    return torch.arange(s, dtype=torch.long, device=token_ids.device).unsqueeze(0) \
        .expand_as(token_ids)


class BertLMHead(MegatronModule):
    """dense -> GeLU -> LayerNorm -> tied vocab-parallel logits + bias."""

    def __init__(self, mpu_vocab_size, hidden_size, init_method, layernorm_epsilon,
                 parallel_output):
        super().__init__()
        args = global_vars.get_args()
        self.bias = torch.nn.Parameter(torch.zeros(mpu_vocab_size))
        tp.set_tensor_model_parallel_attributes(self.bias, True, 0, 1)
        self.parallel_output = parallel_output
        self.dense = get_linear_layer(hidden_size, hidden_size, init_method)
        setattr(self.dense.weight, "sequence_parallel", args.sequence_parallel)
        setattr(self.dense.bias, "sequence_parallel", args.sequence_parallel)
        self.layernorm = MixedFusedLayerNorm(hidden_size, eps=layernorm_epsilon,
                                             sequence_parallel=args.sequence_parallel)
        self.gelu = erf_gelu if args.onnx_safe else torch.nn.functional.gelu

    def forward(self, hidden_states, word_embeddings_weight):
        h = self.layernorm(self.gelu(self.dense(hidden_states)))
        return parallel_lm_logits(h, word_embeddings_weight, self.parallel_output,
                                  bias=self.bias)


def post_language_model_processing(lm_output, pooled_output, lm_head, binary_head, lm_labels,
                                   logit_weights, fp16_lm_cross_entropy):
    lm_logits = lm_head(lm_output, logit_weights)
    binary_logits = binary_head(pooled_output) if binary_head is not None else None
    if lm_labels is None:
        return lm_logits.transpose(0, 1).contiguous(), binary_logits
    labels = lm_labels.transpose(0, 1).contiguous()
    if fp16_lm_cross_entropy and lm_logits.dtype != torch.half:
        raise AssertionError("fp16_lm_cross_entropy requires fp16 logits")
    loss = vocab_parallel_cross_entropy(lm_logits, labels)
    return loss.transpose(0, 1).contiguous(), binary_logits


class BertModel(MegatronModule):
    def __init__(self, num_tokentypes=2, add_binary_head=True, parallel_output=True,
                 pre_process=True, post_process=True, model_type=None):
        super().__init__()
        args = global_vars.get_args()
        if not args.tie_embed_logits:
            raise AssertionError("BERT ties the LM head to the word embeddings")
        self.fp16_lm_cross_entropy = args.fp16_lm_cross_entropy
        self.add_binary_head = add_binary_head
        self.parallel_output = parallel_output
        self.pre_process = pre_process
        self.post_process = post_process
        init_method = init_method_normal(args.init_method_std)
        self.language_model, self._language_model_key = get_language_model(
            num_tokentypes=num_tokentypes, add_pooler=add_binary_head,
            encoder_attn_mask_type=AttnMaskType.padding, init_method=init_method,
            scaled_init_method=scaled_init_method_normal(args.init_method_std, args.num_layers),
            pre_process=pre_process, post_process=post_process, args=args,
            model_type=model_type)
        self.initialize_word_embeddings(init_method_normal, args)
        if post_process:
            self.lm_head = BertLMHead(self.word_embeddings_weight().size(0), args.hidden_size,
                                      init_method, args.layernorm_epsilon, parallel_output)
            self._lm_head_key = "lm_head"
            self.binary_head = None
            if add_binary_head:
                self.binary_head = get_linear_layer(args.hidden_size, 2, init_method)
                self._binary_head_key = "binary_head"

    def set_input_tensor(self, input_tensor):
        self.language_model.set_input_tensor(input_tensor)

    def forward(self, bert_model_input, attention_mask, tokentype_ids=None, lm_labels=None):
        ext_mask = bert_extended_attention_mask(attention_mask)
        lm_output = self.language_model(bert_model_input, bert_position_ids(bert_model_input),
                                        ext_mask, tokentype_ids=tokentype_ids)
        if not self.post_process:
            return lm_output
        pooled = None
        if self.add_binary_head:
            lm_output, pooled = lm_output
        return post_language_model_processing(lm_output, pooled, self.lm_head, self.binary_head,
                                              lm_labels, self.word_embeddings_weight(),
                                              self.fp16_lm_cross_entropy)

    def state_dict_for_save_checkpoint(self, prefix="", keep_vars=False):
        sd = {self._language_model_key: self.language_model.state_dict_for_save_checkpoint(
            prefix=prefix, keep_vars=keep_vars)}
        if self.post_process:
            sd[self._lm_head_key] = self.lm_head.state_dict_for_save_checkpoint(
                prefix=prefix, keep_vars=keep_vars)
            if self.add_binary_head:
                sd[self._binary_head_key] = self.binary_head.state_dict(prefix=prefix,
                                                                        keep_vars=keep_vars)
            if not self.pre_process:
                sd[self._word_embeddings_for_head_key] = self.word_embeddings.state_dict(
                    prefix=prefix, keep_vars=keep_vars)
        return sd

    def load_state_dict(self, state_dict, strict=True):
        self.language_model.load_state_dict(state_dict[self._language_model_key], strict=strict)
        if self.post_process:
            self.lm_head.load_state_dict(state_dict[self._lm_head_key], strict=strict)
            if self.add_binary_head:
                self.binary_head.load_state_dict(state_dict[self._binary_head_key],
                                                 strict=strict)
            if not self.pre_process:
                self.word_embeddings.load_state_dict(
                    state_dict[self._word_embeddings_for_head_key], strict=strict)

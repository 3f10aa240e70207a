"""Decoder-only LM (reference ``megatron/model/gpt_model.py``).

With labels the model returns the per-token vocab-parallel CE loss ``[b, s]``
(fp32); without labels the logits ``[b, s, v/tp]``.
"""
import torch

from .. import global_vars
from ..parallel import tensor as tp
from ..ops.cross_entropy import vocab_parallel_cross_entropy
from .enums import AttnMaskType
from .language_model import get_language_model, parallel_lm_logits
from .module import MegatronModule
from .utils import init_method_normal, scaled_init_method_normal


def post_language_model_processing(lm_output, labels, logit_weights, parallel_output,
                                   fp16_lm_cross_entropy):
    output = parallel_lm_logits(lm_output, logit_weights, parallel_output)
    if labels is None:
        return output.transpose(0, 1).contiguous()
    labels = labels.transpose(0, 1).contiguous()
    if fp16_lm_cross_entropy and output.dtype != torch.half:
        raise AssertionError("fp16_lm_cross_entropy requires fp16 logits")
    # The fused CE kernel reads the bf16/fp16 logits and computes in fp32,
    # numerically identical to the reference's explicit ``output.float()``.
    loss = vocab_parallel_cross_entropy(output, labels)
    return loss.transpose(0, 1).contiguous()


class GPTModel(MegatronModule):
    def __init__(self, num_tokentypes=0, parallel_output=True, pre_process=True,
                 post_process=True, model_type=None):
        args = global_vars.get_args()
        super().__init__(share_word_embeddings=args.tie_embed_logits)
        self.tie_embed_logits = args.tie_embed_logits
        self.parallel_output = parallel_output
        self.pre_process = pre_process
        self.post_process = post_process
        self.fp16_lm_cross_entropy = args.fp16_lm_cross_entropy
        self.language_model, self._language_model_key = get_language_model(
            num_tokentypes=num_tokentypes, add_pooler=False,
            encoder_attn_mask_type=AttnMaskType.causal,
            init_method=init_method_normal(args.init_method_std),
            scaled_init_method=scaled_init_method_normal(args.init_method_std, args.num_layers),
            pre_process=pre_process, post_process=post_process, args=args,
            model_type=model_type)
        if self.tie_embed_logits:
            self.initialize_word_embeddings(init_method_normal, args)

    def set_input_tensor(self, input_tensor):
        self.language_model.set_input_tensor(input_tensor)

    def forward(self, input_ids, position_ids, attention_mask, labels=None, tokentype_ids=None,
                inference_params=None):
        lm_output = self.language_model(input_ids, position_ids, attention_mask,
                                        inference_params=inference_params)
        if not self.post_process:
            return lm_output
        return post_language_model_processing(lm_output, labels, self.word_embeddings_weight(),
                                              self.parallel_output, self.fp16_lm_cross_entropy)

    def state_dict_for_save_checkpoint(self, prefix="", keep_vars=False):
        sd = {self._language_model_key: self.language_model.state_dict_for_save_checkpoint(
            prefix=prefix, keep_vars=keep_vars)}
        if self.post_process and not self.pre_process and self.tie_embed_logits:
            sd[self._word_embeddings_for_head_key] = self.word_embeddings.state_dict(
                prefix=prefix, keep_vars=keep_vars)
        return sd

    def load_state_dict(self, state_dict, strict=True):
        if self.post_process and not self.pre_process and self.tie_embed_logits:
            self.word_embeddings.load_state_dict(state_dict["word_embeddings_for_head"],
                                                 strict=strict)
        if self._language_model_key in state_dict:
            state_dict = state_dict[self._language_model_key]
        self.language_model.load_state_dict(state_dict, strict=strict)

"""Sequence classification head on the BERT encoder
(reference ``megatron/model/classification.py``; used by GLUE-style tasks)."""
import torch

from .. import global_vars
from ..utils.misc import print_rank_last
from .bert_model import bert_extended_attention_mask, bert_position_ids
from .enums import AttnMaskType
from .language_model import get_language_model
from .module import MegatronModule
from .utils import get_linear_layer, init_method_normal, scaled_init_method_normal


class Classification(MegatronModule):
    """Pooled [CLS] -> dropout -> linear ``num_classes`` (key ``classification_head``)."""

    def __init__(self, num_classes, num_tokentypes=2, pre_process=True, post_process=True,
                 model_type=None):
        super().__init__(share_word_embeddings=False)
        args = global_vars.get_args()
        self.num_classes = num_classes
        self.pre_process = pre_process
        self.post_process = post_process
        init_method = init_method_normal(args.init_method_std)
        self.language_model, self._language_model_key = get_language_model(
            num_tokentypes=num_tokentypes, add_pooler=True,
            encoder_attn_mask_type=AttnMaskType.padding, init_method=init_method,
            scaled_init_method=scaled_init_method_normal(args.init_method_std, args.num_layers),
            pre_process=pre_process, post_process=post_process, args=args,
            model_type=model_type)
        if post_process:
            self.classification_dropout = torch.nn.Dropout(args.hidden_dropout)
            self.classification_head = get_linear_layer(args.hidden_size, num_classes,
                                                        init_method)
            self._classification_head_key = "classification_head"

    def set_input_tensor(self, input_tensor):
        self.language_model.set_input_tensor(input_tensor)

    def forward(self, model_input, attention_mask, tokentype_ids=None):
        out = self.language_model(model_input, bert_position_ids(model_input),
                                  bert_extended_attention_mask(attention_mask),
                                  tokentype_ids=tokentype_ids)
        if not self.post_process:
            return out
        _, pooled = out
        logits = self.classification_head(self.classification_dropout(pooled))
        return logits.view(-1, self.num_classes)

    def state_dict_for_save_checkpoint(self, prefix="", keep_vars=False):
        sd = {self._language_model_key: self.language_model.state_dict_for_save_checkpoint(
            prefix=prefix, keep_vars=keep_vars)}
        if self.post_process:
            sd[self._classification_head_key] = self.classification_head.state_dict(
                prefix=prefix, keep_vars=keep_vars)
        return sd

    def load_state_dict(self, state_dict, strict=True):
        self.language_model.load_state_dict(state_dict[self._language_model_key], strict=strict)
        if self.post_process:
            if self._classification_head_key in state_dict:
                self.classification_head.load_state_dict(
                    state_dict[self._classification_head_key], strict=strict)
            else:
                print_rank_last(f"***WARNING*** could not find {self._classification_head_key} "
                                "in the checkpoint, initializing to random")

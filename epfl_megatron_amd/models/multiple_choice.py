"""Multiple-choice head (reference ``megatron/model/multiple_choice.py``; RACE).

Input ``[b, choices, s]`` is folded to ``[b * choices, s]``, each choice is
scored by a 1-unit linear head on the pooled [CLS], and the scores are
reshaped to ``[b, choices]``."""
import torch

from .. import global_vars
from ..utils.misc import print_rank_last
from .bert_model import bert_extended_attention_mask, bert_position_ids
from .enums import AttnMaskType
from .language_model import get_language_model
from .module import MegatronModule
from .utils import get_linear_layer, init_method_normal, scaled_init_method_normal


class MultipleChoice(MegatronModule):
    def __init__(self, num_tokentypes=2, pre_process=True, post_process=True, model_type=None):
        super().__init__(share_word_embeddings=False)
        args = global_vars.get_args()
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
            self.multichoice_dropout = torch.nn.Dropout(args.hidden_dropout)
            self.multichoice_head = get_linear_layer(args.hidden_size, 1, init_method)
            self._multichoice_head_key = "multichoice_head"

    def set_input_tensor(self, input_tensor):
        self.language_model.set_input_tensor(input_tensor)

    def forward(self, model_input, attention_mask, tokentype_ids=None):
        if attention_mask.dim() != 3 or model_input.dim() != 3:
            raise AssertionError("expected [b, choices, s] inputs")
        num_choices = attention_mask.shape[1]
        ids = model_input.view(-1, model_input.size(-1))
        mask = attention_mask.view(-1, attention_mask.size(-1))
        types = None if tokentype_ids is None else tokentype_ids.view(-1, tokentype_ids.size(-1))
        out = self.language_model(ids, bert_position_ids(ids), bert_extended_attention_mask(mask),
                                  tokentype_ids=types)
        if not self.post_process:
            return out
        _, pooled = out
        logits = self.multichoice_head(self.multichoice_dropout(pooled))
        return logits.view(-1, num_choices)

    def state_dict_for_save_checkpoint(self, prefix="", keep_vars=False):
        sd = {self._language_model_key: self.language_model.state_dict_for_save_checkpoint(
            prefix=prefix, keep_vars=keep_vars)}
        if self.post_process:
            sd[self._multichoice_head_key] = self.multichoice_head.state_dict(
                prefix=prefix, keep_vars=keep_vars)
        return sd

    def load_state_dict(self, state_dict, strict=True):
        self.language_model.load_state_dict(state_dict[self._language_model_key], strict=strict)
        if self.post_process:
            if self._multichoice_head_key in state_dict:
                self.multichoice_head.load_state_dict(state_dict[self._multichoice_head_key],
                                                      strict=strict)
            else:
                print_rank_last(f"***WARNING*** could not find {self._multichoice_head_key} in "
                                "the checkpoint, initializing to random")

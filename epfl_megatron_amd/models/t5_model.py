"""T5 encoder-decoder (reference ``megatron/model/t5_model.py``; legacy family).

Encoder and decoder share the (tied) word embedding; the LM head is the tied
vocab-parallel projection plus a ``[v/tp]`` bias (key ``lm_head.bias``).
Masks are bool ``[b, sq, sk]`` with True = masked out (``pretrain_t5.get_batch``
converts the dataset's 1 = keep arrays with ``< 0.5``, as the reference).
"""
import torch

from .. import global_vars
from ..ops.cross_entropy import vocab_parallel_cross_entropy
from ..parallel import tensor as tp
from .enums import AttnMaskType
from .language_model import get_language_model, parallel_lm_logits
from .module import MegatronModule
from .utils import init_method_normal, scaled_init_method_normal


def t5_extended_attention_mask(attention_mask_list):
    """bool ``[b, sq, sk]`` (True = masked) -> ``[b, 1, sq, sk]``; integer masks
    (1 = keep, the dataset's convention) are converted on the way."""
    return [(m if m.dtype == torch.bool else m < 0.5).unsqueeze(1) for m in attention_mask_list]


def t5_position_ids(token_ids):
    s = token_ids.size(1)
    return torch.arange(s, dtype=torch.long, device=token_ids.device).unsqueeze(0) \
        .expand_as(token_ids)


class T5LMHead(MegatronModule):
    def __init__(self, mpu_vocab_size, parallel_output):
        super().__init__()
        self.bias = torch.nn.Parameter(torch.zeros(mpu_vocab_size))
        tp.set_tensor_model_parallel_attributes(self.bias, True, 0, 1)
        self.parallel_output = parallel_output

    def forward(self, hidden_states, word_embeddings_weight):
        return parallel_lm_logits(hidden_states, word_embeddings_weight, self.parallel_output,
                                  bias=self.bias)


class T5Model(MegatronModule):
    def __init__(self, num_tokentypes=0, parallel_output=True, pre_process=True,
                 post_process=True, add_encoder=True, add_decoder=True, model_type=None):
        super().__init__()
        args = global_vars.get_args()
        if not args.tie_embed_logits:
            raise AssertionError("T5 ties the LM head to the word embeddings")
        self.fp16_lm_cross_entropy = args.fp16_lm_cross_entropy
        self.parallel_output = parallel_output
        self.pre_process = pre_process
        self.post_process = post_process
        self.add_encoder = add_encoder
        self.add_decoder = add_decoder
        self.language_model, self._language_model_key = get_language_model(
            num_tokentypes=num_tokentypes, add_pooler=False, add_encoder=add_encoder,
            add_decoder=add_decoder, encoder_attn_mask_type=AttnMaskType.padding,
            decoder_attn_mask_type=AttnMaskType.padding,
            init_method=init_method_normal(args.init_method_std),
            scaled_init_method=scaled_init_method_normal(args.init_method_std, args.num_layers),
            pre_process=pre_process, post_process=post_process, args=args,
            model_type=model_type)
        self.initialize_word_embeddings(init_method_normal, args)
        if post_process and add_decoder:
            self.lm_head = T5LMHead(self.word_embeddings_weight().size(0), parallel_output)
            self._lm_head_key = "lm_head"

    def set_input_tensor(self, input_tensor):
        self.language_model.set_input_tensor(input_tensor)

    def forward(self, encoder_input_ids, decoder_input_ids, encoder_attn_mask, decoder_attn_mask,
                encoder_decoder_attn_mask, tokentype_ids=None, lm_labels=None,
                enc_hidden_states=None):
        enc_mask, dec_mask, enc_dec_mask = t5_extended_attention_mask(
            [encoder_attn_mask, decoder_attn_mask, encoder_decoder_attn_mask])
        lm_output = self.language_model(
            encoder_input_ids, t5_position_ids(encoder_input_ids), enc_mask,
            decoder_input_ids, t5_position_ids(decoder_input_ids), dec_mask, enc_dec_mask,
            tokentype_ids=tokentype_ids, enc_hidden_states=enc_hidden_states)
        if self.post_process and self.add_decoder:
            decoder_output, _ = lm_output
            logits = self.lm_head(decoder_output, self.word_embeddings_weight())
            if lm_labels is None:
                return logits.transpose(0, 1).contiguous()
            if self.fp16_lm_cross_entropy and logits.dtype != torch.half:
                raise AssertionError("fp16_lm_cross_entropy requires fp16 logits")
            loss = vocab_parallel_cross_entropy(logits, lm_labels.transpose(0, 1).contiguous())
            return loss.transpose(0, 1).contiguous()
        if self.add_decoder and not self.add_encoder:
            return lm_output[0]
        return lm_output

    def state_dict_for_save_checkpoint(self, prefix="", keep_vars=False):
        sd = {self._language_model_key: self.language_model.state_dict_for_save_checkpoint(
            prefix=prefix, keep_vars=keep_vars)}
        if self.post_process and self.add_decoder:
            sd[self._lm_head_key] = self.lm_head.state_dict_for_save_checkpoint(
                prefix=prefix, keep_vars=keep_vars)
            if not self.pre_process:
                sd[self._word_embeddings_for_head_key] = self.word_embeddings.state_dict(
                    prefix=prefix, keep_vars=keep_vars)
        return sd

    def load_state_dict(self, state_dict, strict=True):
        self.language_model.load_state_dict(state_dict[self._language_model_key], strict=strict)
        if self.post_process and self.add_decoder:
            self.lm_head.load_state_dict(state_dict[self._lm_head_key], strict=strict)
            if not self.pre_process:
                self.word_embeddings.load_state_dict(
                    state_dict[self._word_embeddings_for_head_key], strict=strict)

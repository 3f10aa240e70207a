"""Dual BERT encoders for retrieval: ICT pretraining and ORQA evaluation
(reference ``megatron/model/biencoder_model.py``; legacy family).

``BiEncoderModel`` holds a query and a context ``PretrainedBertModel`` (or one
shared model); each embeds its input as the [CLS] hidden state, optionally
projected to ``--biencoder_projection_dim``.  TP = PP = 1 only, as in the
reference.
"""
import os

import torch

from .. import global_vars
from ..parallel import state
from ..utils.misc import print_rank_0
from .bert_model import bert_position_ids
from .enums import AttnMaskType
from .language_model import get_language_model
from .module import MegatronModule
from .utils import get_linear_layer, init_method_normal, scaled_init_method_normal


def get_model_provider(only_query_model=False, only_context_model=False,
                       biencoder_shared_query_context_model=False, model_type=None):
    def model_provider(pre_process=True, post_process=True):
        print_rank_0("building Biencoder model ...")
        return biencoder_model_provider(
            only_query_model=only_query_model, only_context_model=only_context_model,
            biencoder_shared_query_context_model=biencoder_shared_query_context_model,
            pre_process=pre_process, post_process=post_process, model_type=model_type)
    return model_provider


def biencoder_model_provider(only_query_model=False, only_context_model=False,
                             biencoder_shared_query_context_model=False, pre_process=True,
                             post_process=True, model_type=None):
    if state.get_tensor_model_parallel_world_size() != 1 or \
            state.get_pipeline_model_parallel_world_size() != 1:
        raise AssertionError("Model parallel size > 1 not supported for ICT")
    # two token types, like the BERT checkpoint the encoders are initialised from
    return BiEncoderModel(num_tokentypes=2, parallel_output=False,
                          only_query_model=only_query_model,
                          only_context_model=only_context_model,
                          biencoder_shared_query_context_model=biencoder_shared_query_context_model,
                          pre_process=pre_process, post_process=post_process,
                          model_type=model_type)


class BiEncoderModel(MegatronModule):
    def __init__(self, num_tokentypes=1, parallel_output=True, only_query_model=False,
                 only_context_model=False, biencoder_shared_query_context_model=False,
                 pre_process=True, post_process=True, model_type=None):
        super().__init__()
        args = global_vars.get_args()
        if only_context_model and only_query_model:
            raise AssertionError("only_query_model and only_context_model are exclusive")
        kw = dict(num_tokentypes=num_tokentypes, parallel_output=parallel_output,
                  pre_process=pre_process, post_process=post_process, model_type=model_type)
        self.biencoder_shared_query_context_model = biencoder_shared_query_context_model
        self.use_context_model = not only_query_model
        self.use_query_model = not only_context_model
        self.biencoder_projection_dim = args.biencoder_projection_dim
        self.query_model = self.context_model = None
        if biencoder_shared_query_context_model:
            self.model = PretrainedBertModel(**kw)
            self._model_key = "shared_model"
            self.query_model = self.context_model = self.model
        else:
            if self.use_query_model:
                self.query_model = PretrainedBertModel(**kw)
                self._query_key = "query_model"
            if self.use_context_model:
                self.context_model = PretrainedBertModel(**kw)
                self._context_key = "context_model"

    def set_input_tensor(self, input_tensor):
        return  # TP = PP = 1 only

    def forward(self, query_tokens, query_attention_mask, query_types, context_tokens,
                context_attention_mask, context_types):
        if not self.use_query_model:
            raise ValueError("Cannot embed query without the query model.")
        if not self.use_context_model:
            raise ValueError("Cannot embed block without the block model.")
        q = self.embed_text(self.query_model, query_tokens, query_attention_mask, query_types)
        c = self.embed_text(self.context_model, context_tokens, context_attention_mask,
                            context_types)
        return q, c

    @staticmethod
    def embed_text(model, tokens, attention_mask, token_types):
        return model(tokens, attention_mask, token_types)

    def state_dict_for_save_checkpoint(self, prefix="", keep_vars=False):
        if self.biencoder_shared_query_context_model:
            return {self._model_key: self.model.state_dict_for_save_checkpoint(
                prefix=prefix, keep_vars=keep_vars)}
        sd = {}
        if self.use_query_model:
            sd[self._query_key] = self.query_model.state_dict_for_save_checkpoint(
                prefix=prefix, keep_vars=keep_vars)
        if self.use_context_model:
            sd[self._context_key] = self.context_model.state_dict_for_save_checkpoint(
                prefix=prefix, keep_vars=keep_vars)
        return sd

    def load_state_dict(self, state_dict, strict=True):
        if self.biencoder_shared_query_context_model:
            self.model.load_state_dict(state_dict[self._model_key], strict=strict)
            return
        if self.use_query_model:
            self.query_model.load_state_dict(state_dict[self._query_key], strict=strict)
        if self.use_context_model:
            self.context_model.load_state_dict(state_dict[self._context_key], strict=strict)

    def init_state_dict_from_bert(self):
        """Iteration-0 ICT init: copy a pretrained BERT ``language_model`` into
        both encoders (and share the query projection with the context side)."""
        from ..checkpointing import (fix_query_key_value_ordering, get_checkpoint_names,
                                     get_checkpoint_tracker_filename, read_metadata, safe_load)
        args = global_vars.get_args()
        if args.bert_load is None:
            print_rank_0("bert_load argument is None")
            return
        tracker = get_checkpoint_tracker_filename(args.bert_load)
        if not os.path.isfile(tracker):
            raise FileNotFoundError("Could not find BERT checkpoint")
        iteration, release = read_metadata(tracker)
        name, _ = get_checkpoint_names(args.bert_load, iteration, False, release=release)
        print_rank_0(f"loading BERT checkpoint {name}")
        sd = safe_load(name)
        version = sd.get("checkpoint_version", 0)
        lm = sd["model"]["language_model"]
        if self.biencoder_shared_query_context_model:
            self.model.language_model.load_state_dict(lm)
            fix_query_key_value_ordering(self.model, version)
            return
        proj = None
        if self.use_query_model:
            self.query_model.language_model.load_state_dict(lm)
            if self.biencoder_projection_dim > 0:
                proj = self.query_model.projection_enc.state_dict()
            fix_query_key_value_ordering(self.query_model, version)
        if self.use_context_model:
            self.context_model.language_model.load_state_dict(lm)
            if proj is not None:
                self.context_model.projection_enc.load_state_dict(proj)
            fix_query_key_value_ordering(self.context_model, version)


class PretrainedBertModel(MegatronModule):
    """BERT encoder whose output is the [CLS] hidden state (+ optional projection)."""

    def __init__(self, num_tokentypes=2, parallel_output=True, pre_process=True,
                 post_process=True, model_type=None):
        super().__init__()
        args = global_vars.get_args()
        self.pad_id = global_vars.get_tokenizer().pad
        self.biencoder_projection_dim = args.biencoder_projection_dim
        self.parallel_output = parallel_output
        self.pre_process = pre_process
        self.post_process = post_process
        init_method = init_method_normal(args.init_method_std)
        self.language_model, self._language_model_key = get_language_model(
            num_tokentypes=num_tokentypes, add_pooler=False,
            encoder_attn_mask_type=AttnMaskType.padding, init_method=init_method,
            scaled_init_method=scaled_init_method_normal(args.init_method_std, args.num_layers),
            pre_process=pre_process, post_process=post_process, args=args,
            model_type=model_type)
        if args.biencoder_projection_dim > 0:
            self.projection_enc = get_linear_layer(args.hidden_size,
                                                   args.biencoder_projection_dim, init_method)
            self._projection_enc_key = "projection_enc"

    def forward(self, input_ids, attention_mask, tokentype_ids=None):
        # attention_mask: bool [b, s, s], True = masked (get_ict_batch converts)
        mask = attention_mask.unsqueeze(1)
        if mask.dtype != torch.bool:
            mask = mask < 0.5
        lm_output = self.language_model(input_ids, bert_position_ids(input_ids), mask,
                                        tokentype_ids=tokentype_ids)
        pooled = lm_output[0, :, :].to(lm_output.dtype)
        if self.biencoder_projection_dim:
            pooled = self.projection_enc(pooled)
        return pooled

    def state_dict_for_save_checkpoint(self, prefix="", keep_vars=False):
        sd = {self._language_model_key: self.language_model.state_dict_for_save_checkpoint(
            prefix=prefix, keep_vars=keep_vars)}
        if self.biencoder_projection_dim > 0:
            sd[self._projection_enc_key] = self.projection_enc.state_dict(prefix=prefix,
                                                                          keep_vars=keep_vars)
        return sd

    def load_state_dict(self, state_dict, strict=True):
        self.language_model.load_state_dict(state_dict[self._language_model_key], strict=strict)
        if self.biencoder_projection_dim > 0:
            self.projection_enc.load_state_dict(state_dict[self._projection_enc_key],
                                                strict=strict)

"""Embedding + transformer stack + LM head (reference ``megatron/model/language_model.py``).

State-dict layout is preserved, including the backward
compatible key remaps on load (``transformer`` -> ``encoder``,
``.attention.`` -> ``.self_attention.``, flat ``word_embeddings.weight``).
"""
import torch
from torch import nn

from .. import global_vars
from ..parallel import state
from ..parallel import tensor as tp
from ..parallel.tensor.layers import _initialize_affine_weight_cpu, _initialize_affine_weight_gpu
from .enums import AttnMaskType, LayerType, PositionEmbeddingType
from .module import MegatronModule
from .transformer import ParallelTransformer
from .utils import get_linear_layer, init_method_normal, scaled_init_method_normal


def parallel_lm_logits(input_, word_embeddings_weight, parallel_output, bias=None):
    """``[s, b, h] x [v/tp, h]^T -> [s, b, v/tp]`` (gathered if not parallel_output)."""
    args = global_vars.get_args()
    if args.async_tensor_model_parallel_allreduce or args.sequence_parallel:
        input_parallel = input_
        model_parallel = state.get_tensor_model_parallel_world_size() > 1
        async_grad_allreduce = args.async_tensor_model_parallel_allreduce and model_parallel \
            and not args.sequence_parallel
    else:
        input_parallel = tp.copy_to_tensor_model_parallel_region(input_)
        async_grad_allreduce = False
    logits = tp.linear_with_grad_accumulation_and_async_allreduce(
        input_parallel, word_embeddings_weight, bias, args.gradient_accumulation_fusion,
        async_grad_allreduce, args.sequence_parallel)
    if parallel_output:
        return logits
    return tp.gather_from_tensor_model_parallel_region(logits)


def get_language_model(num_tokentypes, add_pooler, encoder_attn_mask_type, init_method=None,
                       scaled_init_method=None, add_encoder=True, add_decoder=False,
                       decoder_attn_mask_type=AttnMaskType.causal, pre_process=True,
                       post_process=True, args=None, model_type=None):
    if init_method is None:
        init_method = init_method_normal(args.init_method_std)
    if scaled_init_method is None:
        scaled_init_method = scaled_init_method_normal(args.init_method_std, args.num_layers)
    lm = TransformerLanguageModel(init_method, scaled_init_method, encoder_attn_mask_type,
                                  num_tokentypes=num_tokentypes, add_encoder=add_encoder,
                                  add_decoder=add_decoder,
                                  decoder_attn_mask_type=decoder_attn_mask_type,
                                  add_pooler=add_pooler, pre_process=pre_process,
                                  post_process=post_process, args=args, model_type=model_type)
    return lm, "language_model"


class Pooler(MegatronModule):
    """Dense + tanh over the hidden state at ``sequence_index`` (BERT-style)."""

    def __init__(self, hidden_size, init_method, args):
        super().__init__()
        self.dense = get_linear_layer(hidden_size, hidden_size, init_method)
        self.sequence_parallel = args.sequence_parallel

    def forward(self, hidden_states, sequence_index=0):
        if self.sequence_parallel:
            hidden_states = tp.gather_from_sequence_parallel_region(
                hidden_states, tensor_parallel_output_grad=False)
        return torch.tanh(self.dense(hidden_states[sequence_index, :, :]))


class Embedding(MegatronModule):
    """word (+ absolute position) (+ token-type) embeddings -> ``[s, b, h]``."""

    def __init__(self, hidden_size, vocab_size, max_position_embeddings, embedding_dropout_prob,
                 init_method, num_tokentypes=0):
        super().__init__()
        args = global_vars.get_args()
        self.hidden_size = hidden_size
        self.init_method = init_method
        self.num_tokentypes = num_tokentypes
        self.word_embeddings = tp.VocabParallelEmbedding(
            vocab_size, hidden_size, init_method=init_method, params_dtype=args.params_dtype,
            use_cpu_initialization=bool(args.use_cpu_initialization),
            perform_initialization=args.perform_initialization)
        self._word_embeddings_key = "word_embeddings"
        self.position_embedding_type = args.position_embedding_type
        if self.position_embedding_type == PositionEmbeddingType.absolute:
            self.position_embeddings = nn.Embedding(max_position_embeddings, hidden_size)
            self._position_embeddings_key = "position_embeddings"
            init_method(self.position_embeddings.weight)
        else:
            self.position_embeddings = None
        self._tokentype_embeddings_key = "tokentype_embeddings"
        if num_tokentypes > 0:
            self.tokentype_embeddings = nn.Embedding(num_tokentypes, hidden_size)
            if args.perform_initialization:
                init_method(self.tokentype_embeddings.weight)
        else:
            self.tokentype_embeddings = None
        self.fp32_residual_connection = args.fp32_residual_connection
        self.sequence_parallel = args.sequence_parallel
        self.embedding_dropout = nn.Dropout(embedding_dropout_prob)

    def zero_parameters(self):
        for emb in (self.word_embeddings, self.position_embeddings, self.tokentype_embeddings):
            if emb is not None:
                emb.weight.data.fill_(0)
                emb.weight.shared = True

    def add_tokentype_embeddings(self, num_tokentypes):
        if self.tokentype_embeddings is not None:
            raise Exception("tokentype embeddings is already initialized")
        self.num_tokentypes = num_tokentypes
        self.tokentype_embeddings = nn.Embedding(num_tokentypes, self.hidden_size)
        self.init_method(self.tokentype_embeddings.weight)

    def forward(self, input_ids, position_ids, tokentype_ids=None):
        emb = self.word_embeddings(input_ids)
        if self.position_embeddings is not None:
            emb = emb + self.position_embeddings(position_ids)
        if tokentype_ids is not None:
            if self.tokentype_embeddings is None:
                raise AssertionError("tokentype embeddings are not configured")
            emb = emb + self.tokentype_embeddings(tokentype_ids)
        emb = emb.transpose(0, 1).contiguous()
        if self.fp32_residual_connection:
            emb = emb.float()
        if self.sequence_parallel:
            emb = tp.scatter_to_sequence_parallel_region(emb)
            with tp.get_cuda_rng_tracker().fork():
                emb = self.embedding_dropout(emb)
        else:
            emb = self.embedding_dropout(emb)
        return emb

    def state_dict_for_save_checkpoint(self, prefix="", keep_vars=False):
        sd = {self._word_embeddings_key: self.word_embeddings.state_dict(prefix=prefix,
                                                                         keep_vars=keep_vars)}
        if self.position_embeddings is not None:
            sd[self._position_embeddings_key] = self.position_embeddings.state_dict(
                prefix=prefix, keep_vars=keep_vars)
        if self.num_tokentypes > 0:
            sd[self._tokentype_embeddings_key] = self.tokentype_embeddings.state_dict(
                prefix=prefix, keep_vars=keep_vars)
        return sd

    @staticmethod
    def _sub(state_dict, key):
        if key in state_dict:
            return state_dict[key]
        return {k.split(key + ".")[1]: v for k, v in state_dict.items() if key + "." in k}

    def load_state_dict(self, state_dict, strict=True):
        self.word_embeddings.load_state_dict(self._sub(state_dict, "word_embeddings"),
                                             strict=strict)
        if self.position_embeddings is not None:
            self.position_embeddings.load_state_dict(
                self._sub(state_dict, "position_embeddings"), strict=strict)
        if self.num_tokentypes > 0:
            sub = self._sub(state_dict, "tokentype_embeddings")
            if sub:
                self.tokentype_embeddings.load_state_dict(sub, strict=strict)
            else:
                print("***WARNING*** expected tokentype embeddings in the checkpoint but could "
                      "not find it", flush=True)


class TransformerLanguageModel(MegatronModule):
    def __init__(self, init_method, output_layer_init_method, encoder_attn_mask_type,
                 num_tokentypes=0, add_encoder=True, add_decoder=False,
                 decoder_attn_mask_type=AttnMaskType.causal, add_pooler=False, pre_process=True,
                 post_process=True, args=None, model_type=None):
        super().__init__()
        self.pre_process = pre_process
        self.post_process = post_process
        self.hidden_size = args.hidden_size
        self.num_tokentypes = num_tokentypes
        self.init_method = init_method
        self.add_encoder = add_encoder
        self.encoder_attn_mask_type = encoder_attn_mask_type
        self.add_decoder = add_decoder
        self.decoder_attn_mask_type = decoder_attn_mask_type
        self.add_pooler = add_pooler
        self.encoder_hidden_state = None
        self.flop_estimate = _flop_estimate(args)
        if pre_process:
            self.embedding = Embedding(self.hidden_size, args.padded_vocab_size,
                                       args.max_position_embeddings,
                                       0.0 if args.lima_dropout else args.hidden_dropout,
                                       init_method, num_tokentypes)
            self._embedding_key = "embedding"
        self.encoder = ParallelTransformer(
            init_method, output_layer_init_method, self_attn_mask_type=encoder_attn_mask_type,
            pre_process=pre_process, post_process=post_process, args=args,
            model_type=model_type) if add_encoder else None
        self._encoder_key = "encoder"
        self.decoder = ParallelTransformer(
            init_method, output_layer_init_method, layer_type=LayerType.decoder,
            self_attn_mask_type=decoder_attn_mask_type, pre_process=pre_process,
            post_process=post_process, args=args, model_type=model_type) if add_decoder else None
        self._decoder_key = "decoder"
        if post_process and add_pooler:
            self.pooler = Pooler(self.hidden_size, init_method, args)
            self._pooler_key = "pooler"
        self.tie_embed_logits = args.tie_embed_logits
        if post_process and not self.tie_embed_logits:
            self._lm_key = "lm_head"
            start, end = tp.VocabUtility.vocab_range_from_global_vocab_size(
                args.padded_vocab_size, state.get_tensor_model_parallel_rank(),
                state.get_tensor_model_parallel_world_size())
            rows = end - start
            cpu_init = bool(args.use_cpu_initialization) or not torch.cuda.is_available()
            dev = None if cpu_init else torch.cuda.current_device()
            self.lm_head = nn.Parameter(torch.empty(rows, self.hidden_size,
                                                    dtype=args.params_dtype, device=dev))
            head_init = nn.init.xavier_uniform_ if args.init_method_xavier_uniform \
                else nn.init.xavier_normal_
            if args.perform_initialization:
                # Reference D21: xavier on the TP shard (std depends on TP); kept
                # for bit-compatible init, CPU path uses the full-matrix master.
                if cpu_init:
                    _initialize_affine_weight_cpu(self.lm_head, args.padded_vocab_size,
                                                  self.hidden_size, rows, 0, head_init,
                                                  params_dtype=args.params_dtype)
                else:
                    _initialize_affine_weight_gpu(self.lm_head, head_init, partition_dim=0)
            else:
                tp.set_tensor_model_parallel_attributes(self.lm_head, True, 0, 1)

    def set_input_tensor(self, input_tensor):
        if not isinstance(input_tensor, list):
            input_tensor = [input_tensor]
        if self.add_encoder and self.add_decoder:
            self.encoder.set_input_tensor(input_tensor[0])
        elif self.add_encoder:
            self.encoder.set_input_tensor(input_tensor[0])
        elif self.add_decoder:
            if len(input_tensor) == 2:
                self.decoder.set_input_tensor(input_tensor[0])
                self.encoder_hidden_state = input_tensor[1]
            elif len(input_tensor) == 1:
                self.decoder.set_input_tensor(None)
                self.encoder_hidden_state = input_tensor[0]
            else:
                raise Exception("input_tensor must have either length 1 or 2")
        else:
            raise Exception("Stage must have at least either encoder or decoder")

    def forward(self, enc_input_ids, enc_position_ids, enc_attn_mask, dec_input_ids=None,
                dec_position_ids=None, dec_attn_mask=None, enc_dec_attn_mask=None,
                tokentype_ids=None, inference_params=None, pooling_sequence_index=0,
                enc_hidden_states=None, output_enc_hidden=False):
        enc_in = self.embedding(enc_input_ids, enc_position_ids, tokentype_ids=tokentype_ids) \
            if self.pre_process else None
        if enc_hidden_states is None:
            if self.encoder is not None:
                enc_out = self.encoder(enc_in, enc_attn_mask, inference_params=inference_params,
                                       position_ids=enc_position_ids)
            else:
                enc_out = self.encoder_hidden_state
        else:
            enc_out = enc_hidden_states.to(enc_in.dtype)
        pooled = None
        if self.post_process and self.add_pooler:
            pooled = self.pooler(enc_out, pooling_sequence_index)
        if not self.add_decoder or output_enc_hidden:
            return (enc_out, pooled) if pooled is not None else enc_out
        dec_in = self.embedding(dec_input_ids, dec_position_ids) if self.pre_process else None
        dec_out = self.decoder(dec_in, dec_attn_mask, encoder_output=enc_out,
                               enc_dec_attn_mask=enc_dec_attn_mask,
                               inference_params=inference_params)
        if pooled is not None:
            return dec_out, enc_out, pooled
        return dec_out, enc_out

    def state_dict_for_save_checkpoint(self, prefix="", keep_vars=False):
        sd = {}
        if self.pre_process:
            sd[self._embedding_key] = self.embedding.state_dict_for_save_checkpoint(
                prefix=prefix, keep_vars=keep_vars)
        if self.add_encoder:
            sd[self._encoder_key] = self.encoder.state_dict_for_save_checkpoint(
                prefix=prefix, keep_vars=keep_vars)
        if self.post_process:
            if self.add_pooler:
                sd[self._pooler_key] = self.pooler.state_dict_for_save_checkpoint(
                    prefix=prefix, keep_vars=keep_vars)
            if not self.tie_embed_logits:
                sd[self._lm_key] = self.lm_head.data
        if self.add_decoder:
            sd[self._decoder_key] = self.decoder.state_dict_for_save_checkpoint(
                prefix=prefix, keep_vars=keep_vars)
        return sd

    def load_state_dict(self, state_dict, strict=True):
        if self.pre_process:
            sub = state_dict.get(self._embedding_key)
            if sub is None:
                sub = {k: v for k, v in state_dict.items() if "_embeddings" in k}
            self.embedding.load_state_dict(sub, strict=strict)
        if self.post_process and not self.tie_embed_logits:
            self.lm_head.data.copy_(state_dict["lm_head"])
        if self.add_encoder:
            if self._encoder_key in state_dict:
                sub = state_dict[self._encoder_key]
            elif "transformer" in state_dict:
                sub = state_dict["transformer"]
            else:
                sub = {k.split("transformer.")[1]: v for k, v in state_dict.items()
                       if "transformer." in k}
            sub = {k.replace(".attention.", ".self_attention."): v for k, v in sub.items()}
            self.encoder.load_state_dict(sub, strict=strict)
        if self.post_process and self.add_pooler:
            if "pooler" not in state_dict:
                raise AssertionError("could not find data for pooler in the checkpoint")
            self.pooler.load_state_dict(state_dict[self._pooler_key], strict=strict)
        if self.add_decoder:
            if "decoder" not in state_dict:
                raise AssertionError("could not find data for decoder in the checkpoint")
            self.decoder.load_state_dict(state_dict[self._decoder_key], strict=strict)


def _flop_estimate(args):
    """Rough per-sequence FLOP estimate kept for parity (reference :370-384)."""
    s = args.max_position_embeddings
    ell, v, h = args.num_layers, args.padded_vocab_size, args.hidden_size
    mlp_mult = 64 if args.glu_activation else 16
    per_layer = 6 * s * h * h + 4 * s * s * h + 2 * s * h * h + mlp_mult * s * h * h
    return ell * per_layer + 6 * s * h * v

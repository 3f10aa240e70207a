"""Model enums.

Values match the reference (``megatron/model/enums.py``) because the numeric
values are pickled into checkpoint ``args``; the
checkpoint loader maps the reference module path onto these classes.
"""
import enum


class ModelType(enum.Enum):
    """Whether the model is a single stack or an encoder + decoder pair."""
    encoder_or_decoder = 1
    encoder_and_decoder = 2


class LayerType(enum.Enum):
    """Role of a transformer layer inside the stack."""
    encoder = 1
    decoder = 2


class AttnType(enum.Enum):
    """Self- or cross-attention."""
    self_attn = 1
    cross_attn = 2


class AttnMaskType(enum.Enum):
    """Padding mask (explicit tensor) or implicit causal mask."""
    padding = 1
    causal = 2


class PositionEmbeddingType(enum.Enum):
    """Rotary (RoPE, Meta-interleaved pairs) or learned absolute embeddings."""
    rotary = 1
    absolute = 2

    def __str__(self):
        return self.name


ALL_ENUMS = (ModelType, LayerType, AttnType, AttnMaskType, PositionEmbeddingType)

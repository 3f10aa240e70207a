"""MI355X-native fused operators (autograd wrappers over ``csrc/*.hip``)."""
from .norms import RMSNorm, MixedFusedLayerNorm, rms_norm, layer_norm
from .rope import rope_table, apply_rotary_emb, precompute_freqs
from .attention import flash_attn_qkvpacked, flash_attn_func, attention_ref
from .activations import glu, swiglu, bias_gelu, gelu, GLU_ACTIVATIONS
from .cross_entropy import vocab_parallel_cross_entropy
from .softmax import FusedScaleMaskSoftmax, attention_mask_func

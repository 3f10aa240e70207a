"""Model families: GPT, Llama-1/2, Falcon (+ legacy BERT/T5 encoders)."""
from .enums import ModelType, LayerType, AttnType, AttnMaskType, PositionEmbeddingType
from .module import MegatronModule, Float16Module
from .gpt_model import GPTModel
from .llama_model import LlamaModel
from .falcon_model import FalconModel
from .language_model import get_language_model

"""Model families: GPT, Llama-1/2, Falcon (+ legacy BERT/T5 encoders)."""
from .enums import ModelType, LayerType, AttnType, AttnMaskType, PositionEmbeddingType
from .module import MegatronModule, Float16Module
from .gpt_model import GPTModel
from .llama_model import LlamaModel
from .falcon_model import FalconModel
from .language_model import get_language_model
from .bert_model import BertModel
from .t5_model import T5Model
from .classification import Classification
from .multiple_choice import MultipleChoice
from .biencoder_model import BiEncoderModel, PretrainedBertModel, biencoder_model_provider

"""Tensor/sequence parallelism (reference ``megatron/core/tensor_parallel``)."""
from .layers import (ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding,
                     linear_with_grad_accumulation_and_async_allreduce,
                     param_is_not_tensor_parallel_duplicate,
                     set_tensor_model_parallel_attributes,
                     set_defaults_if_not_set_tensor_model_parallel_attributes,
                     copy_tensor_model_parallel_attributes,
                     fused_glu_mlp_supported, glu_mlp)
from .mappings import (copy_to_tensor_model_parallel_region,
                       gather_from_tensor_model_parallel_region,
                       gather_from_sequence_parallel_region,
                       reduce_from_tensor_model_parallel_region,
                       scatter_to_tensor_model_parallel_region,
                       scatter_to_sequence_parallel_region,
                       reduce_scatter_to_sequence_parallel_region)
from .random import (checkpoint, get_cuda_rng_tracker, model_parallel_cuda_manual_seed,
                     CudaRNGStatesTracker)
from .utils import (split_tensor_along_last_dim, split_tensor_into_1d_equal_chunks,
                    gather_split_1d_tensor, VocabUtility)
from .data import broadcast_data
from ...ops.cross_entropy import vocab_parallel_cross_entropy

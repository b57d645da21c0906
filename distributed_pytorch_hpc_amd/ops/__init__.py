"""CDNA4 operator library (autograd-aware Python front end of csrc/*.hip).

Every op runs the hand-written HIP kernel on GPU tensors (and raises if the native extension is
missing there) and a PyTorch reference implementation on CPU tensors.
"""
from . import _lib
from .activations import GELU, gelu, swiglu, swiglu_reference
from .batchnorm import BatchNormAct2d, batch_norm_act
from .conv import Conv1x1, Conv3x3, StridedConv2d
from .decode import decode_attention, kv_append_
from .attention import attention_reference, flash_attention, flash_bwd, flash_fwd, rope_attention
from .embedding import Embedding, embedding
from .loss import fused_cross_entropy, latitude_weighted_mse, latitude_weights, vocab_parallel_cross_entropy
from .pool import MaxPool2d, max_pool2s2, max_pool3s2
from .norms import LayerNorm, RMSNorm, add_rms_norm, layer_norm, rms_norm, rmsnorm_reference
from .rope import apply_rope, precompute_rope_tables, rope_, rope_reference

native_available = _lib.available

__all__ = [
    "GELU", "gelu", "swiglu", "swiglu_reference", "attention_reference", "flash_attention", "flash_fwd",
    "flash_bwd", "rope_attention", "BatchNormAct2d", "Conv1x1", "Conv3x3", "StridedConv2d", "batch_norm_act", "Embedding", "embedding", "fused_cross_entropy", "latitude_weighted_mse",
    "latitude_weights", "vocab_parallel_cross_entropy", "LayerNorm", "RMSNorm", "add_rms_norm", "layer_norm",
    "rms_norm", "rmsnorm_reference", "apply_rope", "precompute_rope_tables", "rope_", "rope_reference",
    "native_available", "decode_attention", "kv_append_", "MaxPool2d", "max_pool2s2", "max_pool3s2",
]

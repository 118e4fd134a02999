"""bcfl ops: HIP/CDNA4 kernels behind autograd Functions (GPU) with torch references (CPU)."""
from . import rng, ref
from ._native import available as native_available, native, use_native, load_error
from .functional import (bias_dropout_add_layernorm, layernorm, bias_act, varlen_attention,
                         query_subset_attention,
                         embedding_layernorm, rmsnorm, rope, swiglu, cross_entropy, linear, dropout,
                         wgrad, set_wgrad_overlap, wgrad_overlap_enabled, join_wgrad, linear_act,
                         linear_after_act, gemm_supported, lora_linear, lora_swiglu_mlp,
                         xent_stats_, ResidualTap)
from .flat import (adamw_, adamw_multi_, grad_clip_coef, gossip_mix_, weighted_accumulate_, block_sketch, update_stats, scale_, axpby_,
                   delta_round_end_,
                   cast_copy_, merkle_root_sha256, merkle_root_deferred, root_bytes,
                   leaf_digests_sha256)

__all__ = [
    "rng", "ref", "native_available", "native", "use_native", "load_error",
    "bias_dropout_add_layernorm", "layernorm", "bias_act", "varlen_attention", "query_subset_attention",
    "embedding_layernorm", "rmsnorm", "rope", "swiglu", "cross_entropy", "linear", "dropout", "wgrad",
    "set_wgrad_overlap", "wgrad_overlap_enabled", "join_wgrad", "linear_act", "linear_after_act",
    "gemm_supported", "lora_linear", "lora_swiglu_mlp", "xent_stats_", "ResidualTap",
    "adamw_", "adamw_multi_", "grad_clip_coef", "gossip_mix_", "weighted_accumulate_", "block_sketch", "update_stats", "scale_", "axpby_",
    "delta_round_end_",
    "cast_copy_", "merkle_root_sha256", "merkle_root_deferred", "root_bytes", "leaf_digests_sha256",
]
